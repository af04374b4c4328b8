#!/bin/bash
# The side-register HNSW kernel (wv_hnsw_side_kernel) on the C1 graph's
# filtered and tombstoned legs (the bench's shapes: 1M SIFT-shaped rows,
# M = 64, efConstruction = 128, GPU-built; allow lists Bernoulli(p) seed 3 at
# 10 / 50 % over 10000 queries and 1 % over 1000; 1 % of ids tombstoned, seed
# 5, 10000 queries), each over tools/filtered_probe.py: a rocprofv3 kernel
# trace + stats run, then one PMC pass per counter group (no tracing in the
# counter runs).  Writes gpurun_out/pmc_side/pmc_wv_hnsw_side_kernel_<cfg>.json
# keyed to the build (tools/build_hash.py) for bench.py attach_traffic.
set -e
O=gpurun_out/pmc_side; mkdir -p $O
export TMPDIR=/tmp
export WV_BUILD_HASH=$(python3 -c "import sys; sys.path.insert(0, 'tools'); from build_hash import build_hash; print(build_hash('wv_hnsw_side_kernel'))")
for cfg in ${CFGS:-f10 f50 f1 t1}; do
  case $cfg in
    # (the first pass: exact-visited below 40 % eligible, else the lossy
    # pass, whose redo launch is a separate <.., true> dispatch)
    f10) export PROBE_FRACS=0.1 PROBE_TOMB=; KEY=0.1; NQ=10000; KSUB="wv_hnsw_side_kernel<0, 1, 3, 3, true>";;
    f50) export PROBE_FRACS=0.5 PROBE_TOMB=; KEY=0.5; NQ=10000; KSUB="wv_hnsw_side_kernel<0, 1, 3, 3, false>";;
    f1)  export PROBE_FRACS=0.01 PROBE_TOMB=; KEY=0.01; NQ=1000; KSUB="wv_hnsw_side_kernel<0, 1, 3, 3, true>";;
    t1)  export PROBE_FRACS= PROBE_TOMB=0.01; KEY=tomb:0.01; NQ=10000; KSUB="wv_hnsw_side_kernel<0, 1, 3, 3, false>";;
  esac
  D=/tmp/pmc_side_$cfg; rm -rf $D; mkdir -p $D
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 tools/filtered_probe.py 1000000 - > $O/${cfg}_trace.log 2>&1
  i=0
  for set in "FETCH_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $D/p$i -o run -- python3 tools/filtered_probe.py 1000000 - > $O/${cfg}_p$i.log 2>&1 || echo "$cfg pass $i failed rc=$?"
  done
  CFG=$cfg KEY=$KEY NQ=$NQ D=$D KSUB="$KSUB" python3 - <<'PY'
import csv, glob, json, os, statistics
cfg, D, key, nq = os.environ["CFG"], os.environ["D"], os.environ["KEY"], int(os.environ["NQ"])
K, KSUB = "wv_hnsw_side_kernel", os.environ["KSUB"]
vals = {}
for f in sorted(glob.glob(f"{D}/p*/**/run_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if KSUB in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
out = {k: statistics.median(v) for k, v in vals.items()}
avg_ns, calls = None, None
for f in glob.glob(f"{D}/trace/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if KSUB in r["Name"]:
            avg_ns, calls = float(r["AverageNs"]), int(r["Calls"])
af = float(key) if not key.startswith("tomb") else key
js = {"kernel": K, "N": 1000000, "nq": nq, "dim": 128, "data": "sift", "allow_frac": af,
      "avg_kernel_ns": avg_ns, "calls": calls,
      "note": "read = 2*FETCH_SIZE*1024 (gfx950 half-count correction), median over the side-kernel dispatches "
              "of tools/filtered_probe.py (1 warm + 3 timed batches; tools/pmc_side.sh)",
      "source": f"profiles/pmc_wv_hnsw_side_kernel_{cfg}.json (tools/pmc_side.sh)",
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
json.dump(js, open(f"gpurun_out/pmc_side/pmc_wv_hnsw_side_kernel_{cfg}.json", "w"), indent=1)
print(json.dumps(js))
PY
  find $D/trace -name run_kernel_stats.csv -exec cp {} $O/${cfg}_kernel_stats.csv \;
done
