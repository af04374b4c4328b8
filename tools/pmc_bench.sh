#!/bin/bash
# PMC summaries of a bench line's dominant kernel, collected over bench.py
# itself (the build and the shape the line runs), keyed to the build for
# bench.py attach_traffic: a rocprofv3 kernel trace + stats run, then one
# PMC pass per counter group (no tracing in the counter runs; each group
# within the per-block limits: FETCH_SIZE alone, 8 SQ + 1 GRBM).
#   LINE=head  wv_bf_h16_kernel main pass, configs[1] (1M x 128, 10k queries)
#   LINE=c4    wv_bf_h16w_kernel, configs[3] 100 % leg (10M x 768, 1000 queries)
#   LINE=c4_50 / c4_10 / c4_1  the same kernel on the 50 / 10 / 1 % allow-list legs
#   LINE=c5    wv_hnsw_kernel, configs[4] over the 100M corpus (ef 128)
#   LINE=c3t1  wv_hnsw_side_kernel, configs[2]'s line with 1 % of ids tombstoned
# Output: gpurun_out/pmc_bench/<LINE>/ (logs, kernel stats) and
# gpurun_out/pmc_bench/pmc_<kernel>[_<shape>].json; the raw traces and counter
# tables stay in /tmp (a full run's trace exceeds what gpurun merges back);
# the bench logs (with its 30-s heartbeat) are written under gpurun_out.
set -e
LINE=${LINE:-head}
G=gpurun_out/pmc_bench; mkdir -p $G/$LINE
O=/tmp/pmc_bench/$LINE; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
OFF="--no-cpu-baseline --no-corpus-leg --no-group-leg --no-wide-line --steps 5 --warmup 2"
case $LINE in
  head) ARGS="$OFF --no-hnsw-line --no-c3-line --no-c4-line --no-c5-line"
        KNAME=wv_bf_h16_kernel; KSUB="wv_bf_h16_kernel<8, true, false, true>"; SHAPE="1000000 10000 128 uniform"
        OUTJ=pmc_wv_bf_h16_kernel.json; T=300;;
  c4)   ARGS="$OFF --no-hnsw-line --no-c3-line --no-c5-line --c4-fracs 1.0"
        KNAME=wv_bf_h16w_kernel; KSUB="wv_bf_h16w_kernel<false, 128>"; SHAPE="10000000 1000 768 gauss"
        OUTJ=pmc_wv_bf_h16w_kernel_c4.json; T=300;;
  c4_50|c4_10|c4_1)
        F=${LINE#c4_}; FR=$(python3 -c "print({'50': '0.5', '10': '0.1', '1': '0.01'}['$F'])")
        ARGS="$OFF --no-hnsw-line --no-c3-line --no-c5-line --c4-fracs $FR"
        KNAME=wv_bf_h16w_kernel; KSUB="wv_bf_h16w_kernel<false, 128>"; SHAPE="10000000 1000 768 gauss_allow$FR"
        OUTJ=pmc_wv_bf_h16w_kernel_c4_$F.json; T=300;;
  c3t1) # (the tombstoned leg needs the restatement's counts: CPU baseline on, short)
        ARGS="--no-corpus-leg --no-group-leg --no-wide-line --steps 5 --warmup 2 --cpu-seconds 2 --cpu-seconds-t1 1"
        ARGS="$ARGS --no-hnsw-line --no-c4-line --no-c5-line --no-seq-build"
        KNAME=wv_hnsw_side_kernel; KSUB="wv_hnsw_side_kernel<2, 1, 3, 3, false>"; SHAPE="1200000 10000 100 glove"
        AF="tomb:0.01"; OUTJ=pmc_wv_hnsw_side_kernel_c3t1.json; T=300;;
  c5)   ARGS="$OFF --no-hnsw-line --no-c3-line --no-c4-line"
        KNAME=wv_hnsw_kernel; KSUB="wv_hnsw_kernel<0, false, 2>"; SHAPE="100000000 10000 96 sift"
        OUTJ=pmc_wv_hnsw_kernel_c5.json; T=900;;
esac
export KNAME KSUB SHAPE OUTJ O AF
export WV_BUILD_HASH=$(python3 -c "import sys; sys.path.insert(0, 'tools'); from build_hash import build_hash; print(build_hash('$KNAME'))")
timeout -k 10 $T rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py $ARGS > $G/$LINE/trace.log 2>&1
i=0
for set in "FETCH_SIZE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL $T rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 bench.py $ARGS > $G/$LINE/p$i.log 2>&1
done
python3 - <<'PY'
import csv, glob, json, os, statistics
O, ksub, kname = os.environ["O"], os.environ["KSUB"], os.environ["KNAME"]
N, nq, dim, data = os.environ["SHAPE"].split()
vals = {}
for f in sorted(glob.glob(f"{O}/p*/**/run_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if ksub in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
# the median dispatch: the line's timed launches dominate the count
out = {k: statistics.median(v) for k, v in vals.items()}
avg_ns, calls = None, None
for f in glob.glob(f"{O}/trace/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if ksub in r["Name"]:
            avg_ns, calls = float(r["AverageNs"]), int(r["Calls"])
js = {"kernel": kname, "N": int(N), "nq": int(nq), "dim": int(dim), "data": data,
      "avg_kernel_ns": avg_ns, "calls": calls, "build": os.environ.get("WV_BUILD_HASH"),
      "sq": {k: v for k, v in out.items() if k.startswith("SQ_") or k.startswith("GRBM")},
      "note": "median over the dispatches of bench.py's own run of this line (tools/pmc_bench.sh); "
              "read = 2*FETCH_SIZE*1024 (gfx950 half-count correction)",
      "source": "profiles/%s (tools/pmc_bench.sh LINE=%s)" % (os.environ["OUTJ"], os.path.basename(O))}
if os.environ.get("AF"):
    js["allow_frac"] = os.environ["AF"]
if "FETCH_SIZE" in out:
    js["hbm_read_bytes_per_launch"] = js["hbm_bytes_per_launch"] = 2.0 * out["FETCH_SIZE"] * 1024
sq = js["sq"]
mf = sq.get("SQ_INSTS_MFMA") or 0
if mf:
    js["per_mfma"] = {"valu": sq.get("SQ_INSTS_VALU", 0) / mf, "salu": sq.get("SQ_INSTS_SALU", 0) / mf,
                      "lds": sq.get("SQ_INSTS_LDS", 0) / mf}
if sq.get("SQ_WAVE_CYCLES"):
    js["wait_inst_frac"] = sq.get("SQ_WAIT_INST_ANY", 0) / sq["SQ_WAVE_CYCLES"]
if sq.get("GRBM_GUI_ACTIVE") and avg_ns:
    js["effective_clock_ghz"] = sq["GRBM_GUI_ACTIVE"] / 8.0 / avg_ns
if mf and sq.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None and sq.get("GRBM_GUI_ACTIVE"):
    js["mfma_busy_frac"] = sq["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * sq["GRBM_GUI_ACTIVE"] / 8.0)
if avg_ns and js.get("hbm_bytes_per_launch"):
    js["hbm_gbs_measured"] = js["hbm_bytes_per_launch"] / (avg_ns * 1e-9) / 1e9
json.dump(js, open(os.path.join("gpurun_out/pmc_bench", os.environ["OUTJ"]), "w"), indent=1)
print(json.dumps(js))
PY
find $O/trace -name run_kernel_stats.csv -exec cp {} $G/$LINE/kernel_stats.csv \;
