#!/bin/bash
# HNSW search kernel (wv_hnsw_kernel) on the bench's C1 and C3 shapes: a
# rocprofv3 kernel trace + stats, then separate PMC passes (no tracing in the
# counter runs), over `bench.py --workload hnsw` with the concurrency leg, the
# CPU baseline and the ef sweep off (every hnsw dispatch is one 10000-query
# batch at ef=64).  Writes gpurun_out/pmc_hnsw/pmc_wv_hnsw_kernel_<cfg>.json,
# keyed to the build (tools/build_hash.py) for bench.py attach_traffic.
set -e
O=gpurun_out/pmc_hnsw; mkdir -p $O
export TMPDIR=/tmp
export WV_BUILD_HASH=$(python3 -c "import sys; sys.path.insert(0, 'tools'); from build_hash import build_hash; print(build_hash('wv_hnsw_kernel'))")
COMMON="--workload hnsw --no-cpu-baseline --concurrency= --ef-sweep= --steps 5 --warmup 2"
for cfg in ${CFGS:-c1 c3}; do
  case $cfg in
    c1) ARGS="--rows 1000000 --dim 128 --metric l2-squared --data sift";;
    c3) ARGS="--rows 1200000 --dim 100 --metric cosine-dot --data glove";;
  esac
  D=/tmp/pmc_hnsw_$cfg; rm -rf $D; mkdir -p $D
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $COMMON $ARGS > $O/${cfg}_trace.log 2>&1
  i=0
  for set in "FETCH_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $D/p$i -o run -- python3 bench.py $COMMON $ARGS > $O/${cfg}_p$i.log 2>&1 || echo "$cfg pass $i failed rc=$?"
  done
  CFG=$cfg D=$D python3 - <<'PY'
import csv, glob, json, os, statistics
cfg, D = os.environ["CFG"], os.environ["D"]
shape = {"c1": (1000000, 10000, 128, "sift"), "c3": (1200000, 10000, 100, "glove")}[cfg]
vals, grids = {}, {}
for f in sorted(glob.glob(f"{D}/p*/**/run_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "wv_hnsw_kernel" not in r["Kernel_Name"]:
            continue
        key = (r.get("Dispatch_Id"), r["Counter_Name"])
        vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
out = {k: statistics.median(v) for k, v in vals.items()}
avg_ns, calls = None, None
for f in glob.glob(f"{D}/trace/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wv_hnsw_kernel" in r["Name"]:
            avg_ns, calls = float(r["AverageNs"]), int(r["Calls"])
js = {"kernel": "wv_hnsw_kernel", "N": shape[0], "nq": shape[1], "dim": shape[2], "data": shape[3],
      "avg_kernel_ns": avg_ns, "calls": calls,
      "note": "read = 2*FETCH_SIZE*1024 (gfx950 half-count correction), median over the 10000-query ef=64 "
              "dispatches of bench.py --workload hnsw (tools/pmc_hnsw.sh)",
      "source": f"profiles/pmc_wv_hnsw_kernel_{cfg}.json (tools/pmc_hnsw.sh)",
      "sq": {k: v for k, v in out.items() if k.startswith("SQ_") or k.startswith("GRBM")},
      "build": os.environ.get("WV_BUILD_HASH")}
if "FETCH_SIZE" in out:
    js["hbm_read_bytes_per_launch"] = js["hbm_bytes_per_launch"] = 2.0 * out["FETCH_SIZE"] * 1024
sq = js["sq"]
if sq.get("SQ_WAVE_CYCLES"):
    js["wait_inst_frac"] = sq.get("SQ_WAIT_INST_ANY", 0) / sq["SQ_WAVE_CYCLES"]
if sq.get("GRBM_GUI_ACTIVE") and avg_ns:
    js["effective_clock_ghz"] = sq["GRBM_GUI_ACTIVE"] / 8.0 / avg_ns
if avg_ns and js.get("hbm_bytes_per_launch"):
    js["hbm_gbs_measured"] = js["hbm_bytes_per_launch"] / (avg_ns * 1e-9) / 1e9
json.dump(js, open(f"gpurun_out/pmc_hnsw/pmc_wv_hnsw_kernel_{cfg}.json", "w"), indent=1)
print(json.dumps(js))
PY
  find $D/trace -name "run_kernel_stats.csv" -exec cp {} $O/${cfg}_kernel_stats.csv \;
done
