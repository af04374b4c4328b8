"""Summarise a tools/profile.sh run into profiles/ (committed evidence).

    python tools/pmc_summary.py gpurun_out/prof_r01 profiles/r01_exact [--n N --nq NQ --dim D]

Writes <dst>_kernel_stats.csv (rocprofv3 --stats), <dst>_summary.md and, for
the dominant kernel, profiles/pmc_<kernel>.json with HBM bytes per launch:
  FETCH_SIZE is in KiB and on gfx950 counts half the bytes of wide coalesced
  reads (MI355X_MICROARCH.md, HBM section) -> read bytes = 2 * FETCH_SIZE * 1024;
  WRITE_SIZE (KiB) is exact for 16-B stores -> write bytes = WRITE_SIZE * 1024.
"""
import argparse
import csv
import json
import os
import shutil
import statistics


def per_kernel(path, kernel_sub):
    vals = {}
    if not os.path.exists(path):
        return vals
    for r in csv.DictReader(open(path)):
        if kernel_sub in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: statistics.mean(v) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--kernel", default="wv_bf_mfma_kernel")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--nq", type=int, default=10_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--data", default="uniform")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.dst) or ".", exist_ok=True)
    stats = os.path.join(a.src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, a.dst + "_kernel_stats.csv")
    rows = list(csv.DictReader(open(stats)))
    k = next(r for r in rows if a.kernel in r["Name"])
    avg_ns = float(k["AverageNs"])
    fetch = per_kernel(os.path.join(a.src, "pmc_fetch", "run_counter_collection.csv"), a.kernel)
    write = per_kernel(os.path.join(a.src, "pmc_write", "run_counter_collection.csv"), a.kernel)
    sq = per_kernel(os.path.join(a.src, "pmc_sq", "run_counter_collection.csv"), a.kernel)
    rd = 2 * fetch.get("FETCH_SIZE", 0) * 1024
    wr = write.get("WRITE_SIZE", 0) * 1024
    out = {"kernel": a.kernel, "N": a.n, "nq": a.nq, "dim": a.dim, "data": a.data, "avg_kernel_ns": avg_ns,
           "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
           "hbm_bytes_per_launch": rd + wr, "sq": sq,
           "note": "read = 2*FETCH_SIZE*1024 (gfx950 half-count correction), write = WRITE_SIZE*1024"}
    if a.kernel in ("wv_bf_mfma_kernel", "wv_bf_split_kernel"):
        flops = 2.0 * a.dim * a.n * a.nq
        out["algorithmic_tflops"] = flops / avg_ns / 1e3
        if "SQ_VALU_MFMA_BUSY_CYCLES" in sq and "GRBM_GUI_ACTIVE" in sq:
            out["mfma_busy_frac"] = sq["SQ_VALU_MFMA_BUSY_CYCLES"] / (sq["GRBM_GUI_ACTIVE"] * 1024 / 8) \
                if sq["GRBM_GUI_ACTIVE"] else None
    with open(os.path.join(os.path.dirname(a.dst), "pmc_%s.json" % a.kernel), "w") as f:
        json.dump(out, f, indent=1)
    with open(a.dst + "_summary.md", "w") as f:
        f.write("# rocprofv3 summary: %s\n\n" % os.path.basename(a.dst))
        f.write("| kernel | calls | avg ms | share |\n|---|---|---|---|\n")
        for r in rows[:8]:
            f.write("| %s | %s | %.3f | %.2f%% |\n" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e6,
                                                    float(r["Percentage"])))
        f.write("\nDominant kernel `%s`: HBM read %.3f GB, write %.3f GB per launch (PMC, corrected)\n"
                % (a.kernel, rd / 1e9, wr / 1e9))
        for kk, v in sorted(sq.items()):
            f.write("- %s = %.4g\n" % (kk, v))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
