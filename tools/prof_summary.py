"""Summarise rocprofv3 CSV output of a bench.py run into profiles/<round>_*.md.

  python tools/prof_summary.py --stats gpurun_out/prof/bench_kernel_stats.csv --steps 17 \
      [--fetch gpurun_out/pmc_f/..._counter_collection.csv --write ..._counter_collection.csv \
       --traffic-json profiles/r01_gemm_traffic.json] --bench gpurun_out/bench.json \
      > profiles/r01_kernel_stats.md

--steps: how many fwd+bwd+AdamW steps the profiled command executed in total (warm-up +
graph replays + timed + the roofline's recorded step); times per step = totals / steps, except
the GEMM family, whose per-launch average is exact and whose per-step time is per-launch x
launches per step (bench.py's GEMM-only replays add launches that belong to no step).
"""
import argparse
import collections
import csv
import json
import re

CATS = [
    ("GEMM (MFMA template)", r"gemm_kernel<|gemm_p8<|gemm_ps<"),
    ("GEMM split-K reduce", r"k_splitk_reduce"),
    ("fp32 head GEMM", r"k_gemm_f32"),
    ("BatchNorm", r"k_bn_"),
    ("LayerNorm", r"k_ln_"),
    ("attention", r"k_attn_"),
    ("bias-grad colsum / partial reduce", r"k_colsum|k_reduce_partials|k_sum_rows"),
    ("AdamW / step", r"k_adamw|k_step"),
    ("pool / stem / layout", r"k_maxpool|k_avgpool|k_im2col|k_patchify|k_pack|k_cast|k_conv_grad|"
                             r"k_vit|k_concat|k_split|k_gather|k_scatter"),
    ("elementwise / loss", r"k_relu|k_dropout|k_ce_|k_argmax|k_advance"),
    ("memset / copy (runtime)", r"__amd_rocclr|fillBuffer|copyBuffer"),
]


def is_gemm(name):
    """The MFMA GEMM template's kernels: gemm_kernel<...>, the phased gemm_p8<...> and the
    persistent phased gemm_ps<...>."""
    return "gemm_kernel<" in name or "gemm_p8<" in name or "gemm_ps<" in name


def short(name):
    n = name.replace("void dfu::", "").replace("(dfu::GemmArgs)", "")
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*", "", n) if "gemm_kernel" not in n and "gemm_p" not in n else n
    return n.strip()[:70]


def cat(name):
    for c, pat in CATS:
        if re.search(pat, name):
            return c
    return "other"


OPND = ["KM", "MN", "CONV_FWD", "CONV_DGRAD", "CONV_DGRAD_W", "CONV_WGRAD_X"]
EPI = ["BF16", "BF16_RELU", "BF16_GELU", "F32", "F32_RESID", "BF16_DGELU", "BF16_ADD", "F32_ACC",
       "F32_ACC_CONVW", "BF16_STATS", "PATCH", "F32_STATS", "BF16_DSTATS", "X3_GELU", "F16_DUAL",
       "F16_GELU"]


def gemm_label(name):
    m8 = re.search(r"gemm_p(8|s)<(\d+), (\d+), (\d+)(?:, (\d+))?(?:, (true|false))?>", name)
    if m8:
        kind = "phased" if m8.group(1) == "8" else "persistent phased"
        rows = 2 * int(m8.group(5)) if m8.group(5) else 256
        f16 = " fp16" if m8.group(6) == "true" else ""
        return (f"gemm {OPND[int(m8.group(2))]} x {OPND[int(m8.group(3))]} -> "
                f"{EPI[int(m8.group(4))]} {rows}x256 {kind}{f16}")
    m = re.search(r"gemm_kernel<(\d+), (\d+), (\d+), (\d+), (\d+)(?:, (\d+))?(?:, \d+)?>", name)
    if not m:
        return short(name)
    a, b, e, tm, tn = map(int, m.groups()[:5])
    occ = f" x{m.group(6)}/CU" if m.group(6) and m.group(6) != "1" else ""
    return f"gemm {OPND[a]} x {OPND[b]} -> {EPI[e]} {tm}x{tn}{occ}"


def pmc_by_kernel(path, counter):
    per = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            per[r["Kernel_Name"]] += float(r["Counter_Value"])
            disp[r["Kernel_Name"]].add(r["Dispatch_Id"])
    return per, {k: len(v) for k, v in disp.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--traffic-json", help="write the GEMM-family traffic per launch here")
    ap.add_argument("--bench")
    ap.add_argument("--title", default="rocprofv3 --kernel-trace --stats of bench.py")
    ap.add_argument("--trace", help="the run's kernel_trace.csv: also report the GEMM family's "
                                    "per-launch time over bench.py's timed roofline replays")
    ap.add_argument("--replays", type=int, default=3, help="timed replays (bench.py: 3)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.stats)))
    S = a.steps
    gemm_calls = sum(int(r["Calls"]) for r in rows if is_gemm(r["Name"]))
    GS = S  # steps' worth of GEMM launches (the roofline replays add launches)
    if a.bench:
        b = json.loads(open(a.bench).read().strip().splitlines()[-1])
        GS = gemm_calls / b["roofline"]["launches_per_step"]

    def per_step(r):
        n = r["Name"]
        return GS if (is_gemm(n) or "k_splitk_reduce" in n) else S
    total = sum(float(r["TotalDurationNs"]) / 1e6 / per_step(r) for r in rows)
    print(f"# {a.title}\n")
    print("Kernel durations are summed per step; the encoders run on two streams, so the sum "
          "exceeds the step's wall time (and the profiler itself reduces the overlap).\n")
    print(f"Source: `{a.stats}`; {S} steps executed by the profiled command "
          f"(GEMM launches: {GS:.2f} steps' worth, incl. bench.py's roofline replays); kernel time "
          f"**{total:.3f} ms per step**.\n")
    if a.bench:
        b = json.loads(open(a.bench).read().strip().splitlines()[-1])
        rf = b["roofline"]
        print(f"bench line of the same command: {b['value']} {b['unit']}, {b['ms_per_step']} ms/step; "
              f"GEMM roofline achieved {rf['achieved']} TFLOP/s ({rf['frac'] * 100:.1f}% of "
              f"{rf['peak']}), avg launch {rf['avg_launch_us']} us over "
              f"{rf['launches_per_step']} launches/step.\n")
    cats = collections.defaultdict(float)
    for r in rows:
        cats[cat(r["Name"])] += float(r["TotalDurationNs"]) / 1e6 / per_step(r)
    print("## Per category (ms per step)\n\n| category | ms/step | share |\n|---|---:|---:|")
    for c, v in sorted(cats.items(), key=lambda kv: -kv[1]):
        print(f"| {c} | {v:.3f} | {100 * v / total:.1f}% |")
    g = [r for r in rows if is_gemm(r["Name"]) or "k_splitk_reduce" in r["Name"]]
    gl = [r for r in g if is_gemm(r["Name"])]
    g_ns = sum(float(r["TotalDurationNs"]) for r in g)
    g_calls = sum(int(r["Calls"]) for r in gl)
    per_launch_us = g_ns / 1e3 / g_calls
    print(f"\nGEMM family (gemm_kernel + its split-K reductions): {g_calls} launches, "
          f"**{per_launch_us:.2f} us per launch** (bench.py's `avg_launch_us` measures the same "
          f"launches with HIP events around back-to-back replays).\n")
    if a.trace and a.bench:
        b = json.loads(open(a.bench).read().strip().splitlines()[-1])
        L = b["roofline"]["launches_per_step"]
        ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                    for r in csv.DictReader(open(a.trace)))
        fam = [k for k in ks if is_gemm(k[2]) or "k_splitk_reduce" in k[2]]
        gi = [i for i, k in enumerate(fam) if is_gemm(k[2])]
        first = gi[-a.replays * L]  # the first GEMM of the timed replays (the last ones traced)
        win = fam[first:]
        busy = sum(e - st for st, e, _ in win) / 1e3 / (a.replays * L)
        wall = (win[-1][1] - win[0][0]) / 1e3 / (a.replays * L)
        print(f"Over bench.py's {a.replays} timed roofline replays in this trace (the same "
              f"{L} launches back to back on one stream, as `avg_launch_us` times them): "
              f"**{busy:.2f} us per launch** of kernel time, {wall:.2f} us per launch from the "
              f"first start to the last end (bench line: {b['roofline']['avg_launch_us']} us).\n")
    if a.fetch and a.write:
        fetch, fn = pmc_by_kernel(a.fetch, "FETCH_SIZE")
        write, wn = pmc_by_kernel(a.write, "WRITE_SIZE")
        gk = [k for k in fetch if is_gemm(k) or "k_splitk_reduce" in k]
        launches = sum(fn[k] for k in gk if is_gemm(k))
        fb = sum(fetch[k] for k in gk) * 1024 * 2 / launches  # gfx950: FETCH_SIZE = 1/2 of 16-B streams
        wb = sum(write.get(k, 0.0) for k in gk) * 1024 / launches
        print(f"HBM traffic of the GEMM family (PMC, separate --pmc FETCH_SIZE and --pmc WRITE_SIZE "
              f"passes over {launches} launches; FETCH_SIZE x 2 per the gfx950 correction, "
              f"WRITE_SIZE x 1, KiB -> B): read {fb / 1e6:.2f} MB + write {wb / 1e6:.2f} MB = "
              f"**{(fb + wb) / 1e6:.2f} MB per launch**.\n")
        if a.traffic_json:
            with open(a.traffic_json, "w") as f:
                json.dump({"bytes_per_launch": fb + wb, "read_bytes_per_launch": fb,
                           "write_bytes_per_launch": wb, "launches_sampled": launches,
                           "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE: {a.fetch}, {a.write}",
                           "correction": "FETCH_SIZE*2*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM)"},
                          f, indent=1)
    print("## Top kernels\n\n| kernel | calls/step | avg us | ms/step | share |\n|---|---:|---:|---:|---:|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]) / per_step(r))[:40]:
        t = float(r["TotalDurationNs"]) / 1e6 / per_step(r)
        print(f"| `{gemm_label(r['Name'])}` | {int(r['Calls']) / per_step(r):.1f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {t:.3f} | {100 * t / total:.1f}% |")


if __name__ == "__main__":
    main()
