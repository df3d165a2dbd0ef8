#!/bin/bash
# GPU-box recipe (round 4, re-entry): full GPU suite, smoke(), default bench,
# its kernel stats, then the K2 MFMA prototype and the host-MD5 probe.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4g}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/k2_mfma_probe.hip -o $OUT/k2_mfma_probe > $OUT/mfma_build.log 2>&1
timeout -k 10 120 $OUT/k2_mfma_probe > $OUT/mfma_probe.log 2>&1
timeout -k 10 200 python -u tools/md5_host_probe.py > $OUT/md5_host.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 $R/bench.py --no-cpu-baseline --no-t2t > "$OUT/prof.log" 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d "$OUT/prof_mfma" -o run --output-format csv \
    -- $OUT/k2_mfma_probe > "$OUT/prof_mfma.log" 2>&1
cd "$R"
for L in product d3 d4 d5 d6 d7; do
  if [ $L = product ]; then
    timeout -k 10 200 python -u tools/dec_probe.py --tag product >> $OUT/dec_probe.log 2>&1
  else
    ATGPU_LIB=$R/expgpu/libatgpu_$L.so timeout -k 10 200 python -u tools/dec_probe.py --tag $L >> $OUT/dec_probe.log 2>&1
  fi
done
