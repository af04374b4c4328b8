mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
A="--workload hnsw --rows 1000000 --ef 64 --graph-cache /tmp/g1m.npz --steps 3 --warmup 1"
timeout -k 10 900 python -u bench.py $A --cpu-seconds 5 > gpurun_out/hb_default.log 2>&1 || exit $?
tail -1 gpurun_out/hb_default.log | cut -c1-1500
for kb in 8 16 20; do
  WV_HNSW_WAVE_KB=$kb timeout -k 10 300 python -u bench.py $A --no-cpu-baseline > gpurun_out/hb_$kb.log 2>&1 || exit $?
  echo "kb=$kb $(tail -1 gpurun_out/hb_$kb.log | grep -o '"kernel_ms": [0-9.]*')"
done
