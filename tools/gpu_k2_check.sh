set -e -o pipefail
mkdir -p gpurun_out/r6bi
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hl_range.py tests/test_gpu_flac.py tests/test_gpu_k2_packed.py > gpurun_out/r6bi/pytest.log 2>&1
bash tools/gpu_k2_profile.sh r6bi
