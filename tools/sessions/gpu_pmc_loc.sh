#!/bin/bash
# L2 behaviour of the brute-force kernel per locality mode: TCC hit/miss and
# FETCH_SIZE (separate passes), plus LDS/SQ counters for the default mode.
export TMPDIR=/tmp
OUT=gpurun_out/pmc_loc; mkdir -p $OUT
A="--no-cpu-baseline --steps 2 --warmup 1"
for L in 3 0; do
  WV_BF_LOCALITY=$L timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/hit_$L -o run -- python3 bench.py $A > $OUT/hit_$L.log 2>&1 || exit $?
  WV_BF_LOCALITY=$L timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$L -o run -- python3 bench.py $A > $OUT/fetch_$L.log 2>&1 || exit $?
done
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/sq -o run -- python3 bench.py $A > $OUT/sq.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr --output-format csv -d $OUT/tcp -o run -- python3 bench.py $A > $OUT/tcp.log 2>&1
python3 - <<'PY'
import csv, glob, statistics, collections
for f in sorted(glob.glob("gpurun_out/pmc_loc/*/*counter_collection.csv")):
    v = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "wv_bf_mfma" in r["Kernel_Name"]:
            v[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f.split("/")[2], {k: "%.4g" % statistics.mean(x) for k, x in v.items()})
PY
