#!/bin/bash
# f16 key pass on the harness (build/h16/abl_base, tools/h16_ablate.sh)
# (KNAME=wv_bf_h16w_kernel KSUB=wv_bf_h16w_kernel N=1250000 NQ=1000 D=768: the
# wide pass on the C4 shape):
# rocprofv3 kernel trace + stats, then separate PMC passes (no tracing in
# the counter runs).  Output under gpurun_out/pmc_h16/.
set -e
O=gpurun_out/pmc_h16; mkdir -p $O
export TMPDIR=/tmp
export WV_BUILD_HASH=${WV_BUILD_HASH:-$(python3 tools/build_hash.py)}
B=${B:-build/h16/abl_base}
ARGS="${N:-1000000} ${NQ:-10000} ${D:-128} pmc"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B $ARGS > $O/trace.log 2>&1
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_WAVES" \
           "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- $B $ARGS > $O/p$i.log 2>&1 || echo "pass $i failed rc=$?"
done
python3 - <<'PY'
import csv, glob, statistics, json, os
out = {}
for f in sorted(glob.glob("gpurun_out/pmc_h16/p*/run_counter_collection.csv")):
    vals = {}
    for r in csv.DictReader(open(f)):
        if os.environ.get("KSUB", "wv_bf_h16_kernel<8, true, false, true>") in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in vals.items():
        out[k] = statistics.mean(v)
for f in glob.glob("gpurun_out/pmc_h16/trace/run_kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:70], r["Calls"], r["AverageNs"])
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/pmc_h16/summary.json", "w"), indent=1)
# the bench's roofline.traffic source (bench.py attach_traffic): HBM bytes per
# launch of the key pass, FETCH_SIZE doubled (gfx950 half-count correction)
import os
avg_ns = None
for f in glob.glob("gpurun_out/pmc_h16/trace/run_kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if os.environ.get("KSUB", "wv_bf_h16_kernel<8, true, false, true>") in r["Name"]:
            avg_ns = float(r["AverageNs"])
if "FETCH_SIZE" in out:
    rd = 2.0 * out["FETCH_SIZE"] * 1024
    kname = os.environ.get("KNAME", "wv_bf_h16_kernel")
    js = {"kernel": kname, "N": int(os.environ.get("N", 1000000)), "nq": int(os.environ.get("NQ", 10000)),
          "dim": int(os.environ.get("D", 128)), "data": "uniform", "avg_kernel_ns": avg_ns,
          "hbm_read_bytes_per_launch": rd, "hbm_bytes_per_launch": rd,
          "algorithmic_bytes_per_launch": None,
          "sq": {k: v for k, v in out.items() if k.startswith("SQ_") or k.startswith("GRBM")},
          "note": "read = 2*FETCH_SIZE*1024 (gfx950 half-count correction); U[0,1) corpus/queries of the "
                  "tools/h16_ablate.cpp harness (same shape as bench.py's configs[1]); write traffic is the "
                  "candidate lists only (not collected)",
          "source": "profiles/pmc_%s.json (tools/pmc_h16.sh)" % kname}
    sq = js["sq"]
    mf = sq.get("SQ_INSTS_MFMA") or 0
    if mf:
        js["per_mfma"] = {"valu": sq.get("SQ_INSTS_VALU", 0) / mf, "salu": sq.get("SQ_INSTS_SALU", 0) / mf,
                          "lds": sq.get("SQ_INSTS_LDS", 0) / mf}
    if sq.get("SQ_WAVE_CYCLES"):
        js["wait_inst_frac"] = sq.get("SQ_WAIT_INST_ANY", 0) / sq["SQ_WAVE_CYCLES"]
        js["wait_any_frac"] = sq.get("SQ_WAIT_ANY", 0) / sq["SQ_WAVE_CYCLES"]
    if sq.get("GRBM_GUI_ACTIVE") and avg_ns:
        js["effective_clock_ghz"] = sq["GRBM_GUI_ACTIVE"] / 8.0 / avg_ns
    if mf and sq.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None and sq.get("GRBM_GUI_ACTIVE"):
        # MFMA pipe busy share: busy cycles summed over SIMDs / (SIMDs x cycles)
        js["mfma_busy_frac"] = sq["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * sq["GRBM_GUI_ACTIVE"] / 8.0)
    js["build"] = os.environ.get("WV_BUILD_HASH")
    json.dump(js, open("gpurun_out/pmc_h16/pmc_%s.json" % kname, "w"), indent=1)
PY
