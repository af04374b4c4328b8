#!/bin/bash
# Rehearse the N-rank bench path on a one-GPU box: N=1 (reference) then N=2
# and N=4 ranks sharing cuda:0 with the gloo backend; the merged ids/dists of
# every N must equal N=1's bit for bit (exact mode).
mkdir -p gpurun_out
A="--steps 2 --warmup 1 --no-cpu-baseline --rows ${RN:-200000} --nq 2000"
timeout -k 10 300 python -u bench.py $A --dump-ids /tmp/ids1.npz > gpurun_out/rank1.log 2>&1 || exit $?
tail -1 gpurun_out/rank1.log | cut -c1-300
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n $A --dist-backend gloo --dump-ids /tmp/ids$n.npz \
    > gpurun_out/rank$n.log 2>&1 || exit $?
  tail -1 gpurun_out/rank$n.log | cut -c1-300
  python - <<PY || exit 1
import numpy as np
a, b = np.load("/tmp/ids1.npz"), np.load("/tmp/ids$n.npz")
same = (a["ids"] == b["ids"]).all() and (a["dists"].view(np.uint32) == b["dists"].view(np.uint32)).all()
print("N=$n merged result identical to N=1:", bool(same))
raise SystemExit(0 if same else 1)
PY
done
