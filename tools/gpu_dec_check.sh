# decoder GPU tests, then the decode leg of the bench in each frame-hypothesis
# mode (0 off, 1 default, 2 self-check), twice
set -e
mkdir -p gpurun_out/deccheck
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_decode_hypothesis.py tests/test_gpu_decode.py tests/test_gpu_decoder_stream.py \
  tests/test_gpu_callers.py > gpurun_out/deccheck/pytest.log 2>&1 || { tail -30 gpurun_out/deccheck/pytest.log; exit 1; }
tail -1 gpurun_out/deccheck/pytest.log
bash tools/gpu_dec_spec.sh
