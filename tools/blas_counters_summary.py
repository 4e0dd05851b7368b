"""hipBLASLt vs dfu side by side from tools/blas_counters.sh output.

  python tools/blas_counters_summary.py gpurun_out/blasctr > profiles/r16_blas_counters.md

Per case and library: the unprofiled time, then per GEMM dispatch (means over the dispatches of
the --pmc runs): clock (GRBM_GUI_ACTIVE / 8 XCDs / time), MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES /
(active cycles x 1024 SIMDs)), the wave-cycle shares parked on s_waitcnt / barriers
(SQ_WAIT_ANY), issue-stalled (SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY), waves per
dispatch (SQ_WAVE_CYCLES / SQ_BUSY_CYCLES is not a count; the launch shape is from the kernel
trace), LDS instructions and VALU instructions per MFMA, and the LDS bank-conflict share.
"""
import csv
import glob
import os
import re
import sys

SIMDS, XCDS = 1024, 8


def counters(d, pat):
    per = {}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            if not re.search(pat, r.get("Kernel_Name", "")):
                continue
            k = (fn, int(r["Dispatch_Id"]))
            per.setdefault(k, {}).setdefault(r["Counter_Name"], 0.0)
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        return {}
    keys = set().union(*per.values())
    return {c: sum(v.get(c, 0.0) for v in per.values()) / len(per) for c in keys}


def launch(d):
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            if "Cijk" in r["Kernel_Name"]:
                m = re.search(r"MT(\d+x\d+x\d+)", r["Kernel_Name"])
                sk = re.search(r"_SK(\d+)", r["Kernel_Name"])
                wgs = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
                return (f"MT{m.group(1) if m else '?'}{' stream-K' if sk else ''}, "
                        f"{int(r['Workgroup_Size_X']) // 64} waves/WG, {wgs} WGs, "
                        f"LDS {int(r['LDS_Block_Size']) // 1024} KiB, VGPR {r['VGPR_Count']}")
    return ""


def main():
    root = sys.argv[1]
    times = {}
    for ln in open(os.path.join(root, "times.txt")):
        m = re.match(r"blas (\S+) \S+: ([\d.]+) us (\d+) TFLOP/s", ln.strip())
        if m:
            times[(m.group(1), "blas")] = (float(m.group(2)), float(m.group(3)))
        m = re.match(r"(\S+) tile (\d+): ([\d.]+) us\s+(\d+) TFLOP/s", ln.strip())
        if m:
            times[(m.group(1), "gemm")] = (float(m.group(3)), float(m.group(4)))
    print("# hipBLASLt (yardstick only) vs the dfu GEMM on the ViT shapes, rocprofv3 --pmc\n")
    print(__doc__.split("\n\n", 1)[1].strip() + "\n")
    print("| case | library | us | TFLOP/s | clock GHz | MFMA busy | wait_any | wait_inst | active "
          "| LDS ins / MFMA | VALU ins / MFMA | SALU ins / MFMA | LDS conflict | kernel |")
    print("|---|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---|")
    cases = sorted({c for c, _ in times}, key=lambda c: list(times).index((c, "blas")))
    for case in cases:
        for lib, pat, name in (("blas", r"Cijk", "hipBLASLt"), ("gemm", r"gemm", "dfu")):
            if (case, lib) not in times:
                continue
            us, tf = times[(case, lib)]
            a = counters(os.path.join(root, f"{case}_{lib}_a"), pat)
            b = counters(os.path.join(root, f"{case}_{lib}_b"), pat)
            if not a:
                continue
            act = a["GRBM_GUI_ACTIVE"] / XCDS
            wc = a["SQ_WAVE_CYCLES"]
            mf = max(b.get("SQ_INSTS_MFMA", 1.0), 1.0)
            conf = b.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(b.get("SQ_LDS_IDX_ACTIVE", 1.0), 1.0)
            kern = launch(os.path.join(root, f"{case}_blas_kt")) if lib == "blas" else \
                "persistent phased 256x256, 8 waves/WG, 256 WGs (tuned plan)"
            print(f"| {case} | {name} | {us:.1f} | {tf:.0f} | {act / us / 1e3:.2f} | "
                  f"{a['SQ_VALU_MFMA_BUSY_CYCLES'] / (act * SIMDS) * 100:.1f}% | "
                  f"{a['SQ_WAIT_ANY'] / wc * 100:.1f}% | {a['SQ_WAIT_INST_ANY'] / wc * 100:.1f}% | "
                  f"{a['SQ_ACTIVE_INST_ANY'] / wc * 100:.1f}% | {b.get('SQ_INSTS_LDS', 0) / mf:.2f} | "
                  f"{b.get('SQ_INSTS_VALU', 0) / mf:.2f} | {b.get('SQ_INSTS_SALU', 0) / mf:.2f} | "
                  f"{conf:.3f} | {kern} |")


if __name__ == "__main__":
    main()
