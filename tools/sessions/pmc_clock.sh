#!/bin/bash
# MFMA busy and effective clock of the f16 key pass binaries (one PMC pass each).
set -e
export TMPDIR=/tmp WV_ABLATE_NO_FALLBACK=1
O=gpurun_out/pmc_clock; mkdir -p $O
for v in ${VARIANTS:-base pure_nolds}; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT \
      --kernel-trace --output-format csv -d $O/$v -o run -- build/h16/abl_$v 1000000 10000 128 $v > $O/$v.log 2>&1 || echo "$v failed"
done
python3 - <<'PY'
import csv, glob, statistics, os
for d in sorted(glob.glob("gpurun_out/pmc_clock/*/")):
    v = os.path.basename(d.rstrip("/"))
    vals, durs = {}, []
    for r in csv.DictReader(open(d + "run_counter_collection.csv")):
        if "h16_kernel<8, true, false>" in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for r in csv.DictReader(open(d + "run_kernel_trace.csv")):
        if "h16_kernel<8, true, false>" in r["Kernel_Name"]:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    m = {k: statistics.mean(x) for k, x in vals.items()}
    t = statistics.mean(durs) if durs else float("nan")
    clk = m["GRBM_GUI_ACTIVE"] / 8 / t if durs else float("nan")
    busy = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8)
    print(f"{v:12s} kernel {t*1e3:.3f} ms  clock {clk/1e9:.2f} GHz  MFMA busy {busy:.3f}  "
          f"wait_any {m['SQ_WAIT_ANY']/m['SQ_WAVE_CYCLES']:.3f}  wait_inst {m['SQ_WAIT_INST_ANY']/m['SQ_WAVE_CYCLES']:.3f}  "
          f"active {m['SQ_ACTIVE_INST_ANY']/m['SQ_WAVE_CYCLES']:.3f}")
PY
