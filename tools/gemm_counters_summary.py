"""MFMA-utilisation table of single GEMM shapes from tools/gemm_counters_r3.sh output.

  python tools/gemm_counters_summary.py gpurun_out/ctr [gpurun_out/actr] > profiles/r21_gemm_counters.md

Per case (tools/gemm_one.py, the library's own plan): the unprofiled time and TFLOP/s, then per
GEMM dispatch of the two --pmc passes (averaged over the 6 dispatches of each run):
  * clock      = GRBM_GUI_ACTIVE / 8 XCDs / unprofiled time;
  * MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): the fraction of
                 the kernel's active cycles each SIMD's matrix pipe was busy (MfmaUtil);
  * MFMA ideal = algorithmic FLOPs / 1024 (v_mfma_f32_16x16x32_bf16: 16 busy cycles per 16384
                 FLOPs, MI355X_MICROARCH.md) over the same cycle budget -- what the busy share
                 would be with no padding or re-issued work;
  * waits      = SQ_WAIT_ANY (parked on s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue stalls)
                 and SQ_ACTIVE_INST_ANY as shares of SQ_WAVE_CYCLES;
  * LDS        = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES, and
                 SQ_INSTS_LDS / SQ_INSTS_MFMA.
With a second directory (tools/attn_counters.sh output) the attention kernels follow (counters
only).
"""
import csv
import glob
import os
import re
import sys

SIMDS = 1024  # 256 CUs x 4
XCDS = 8


def dispatch_counters(d, pat="gemm"):
    """{counter: mean over the dispatches whose kernel name contains pat} of one --pmc run
    directory."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = {}
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name", "")
                if pat not in name:
                    continue
                k = (fn, int(r["Dispatch_Id"]))
                per.setdefault(k, {}).setdefault(r["Counter_Name"], 0.0)
                per[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        return {}
    keys = set().union(*per.values())
    return {c: sum(v.get(c, 0.0) for v in per.values()) / len(per) for c in keys}


def main():
    root = sys.argv[1]
    times = {}
    for ln in open(os.path.join(root, "times.txt")):
        m = re.match(r"(\S+) tile (\d+): ([\d.]+) us\s+(\d+) TFLOP/s", ln.strip())
        if m:  # run directories: <case>_t<tile>_{a,b} (tools/gemm_counters.sh)
            times[f"{m.group(1)}_t{m.group(2)}"] = (float(m.group(3)), float(m.group(4)))
    print("# MFMA utilisation of the step's top GEMM shapes (rocprofv3 --pmc, one MI355X)\n")
    print(__doc__.split("\n\n", 1)[1].strip() + "\n")
    print("| case | us | TFLOP/s | % bf16 peak | clock GHz | MFMA busy | MFMA ideal | wait_any | "
          "wait_inst | active | LDS conflict/active | LDS issue stall | LDS inst per MFMA |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for case, (us, tf) in times.items():
        a = dispatch_counters(os.path.join(root, case + "_a"))
        b = dispatch_counters(os.path.join(root, case + "_b"))
        if not a:
            continue
        rows(case, us, tf, a, b)
    if len(sys.argv) > 2:  # tools/attn_counters.sh output: the attention kernels (no time here)
        for pat in ("k_attn_fwd", "k_attn_bwd"):
            a = dispatch_counters(os.path.join(sys.argv[2], "a"), pat)
            b = dispatch_counters(os.path.join(sys.argv[2], "b"), pat)
            if a:
                rows(pat, None, None, a, b)


def rows(case, us, tf, a, b):
    if True:
        act = a["GRBM_GUI_ACTIVE"] / XCDS
        busy = a["SQ_VALU_MFMA_BUSY_CYCLES"] / (act * SIMDS)
        wc = a["SQ_WAVE_CYCLES"]
        lds_c = b.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(b.get("SQ_LDS_IDX_ACTIVE", 1.0), 1.0)
        lds_w = a.get("SQ_WAIT_INST_LDS", 0.0) / wc if wc else 0.0
        per_mfma = b.get("SQ_INSTS_LDS", 0.0) / max(b.get("SQ_INSTS_MFMA", 1.0), 1.0)
        if us is None:
            t = "| — | — | — | — "
        else:
            flops = tf * 1e12 * us * 1e-6
            ideal = flops / 1024 / (act * SIMDS)
            t = (f"| {us:.1f} | {tf:.0f} | {tf / 2500 * 100:.1f}% | {act / us / 1e3:.2f} | "
                 f"{busy * 100:.1f}% | {ideal * 100:.1f}% ")
            busy = None
        print(f"| {case} {t}" + (f"| {busy * 100:.1f}% | — " if busy is not None else "") +
              f"| {a['SQ_WAIT_ANY'] / wc * 100:.1f}% | "
              f"{a['SQ_WAIT_INST_ANY'] / wc * 100:.1f}% | {a['SQ_ACTIVE_INST_ANY'] / wc * 100:.1f}% | "
              f"{lds_c:.3f} | {lds_w * 100:.1f}% | {per_mfma:.2f} |")


if __name__ == "__main__":
    main()
