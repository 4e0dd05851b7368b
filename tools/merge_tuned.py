"""Merge gemm_tune.py outputs into dfu-multimodal_amd/csrc/gemm_tuned.inc.
  python tools/merge_tuned.py NEW.inc [--only-tiles 10,11] [--new-only]
--only-tiles: replace an existing entry only when the new plan uses one of these tiles (a tile
added since the table was tuned); --new-only: add shapes the table lacks, keep every existing
entry (e.g. the bf16x3 forward's tripled-K shapes)."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "dfu-multimodal_amd", "csrc", "gemm_tuned.inc")


def parse(path):
    out, order = {}, []
    for ln in open(path):
        m = re.match(r"\s*\{([-\d, ]+)\},\s*(//.*)?$", ln.rstrip("\n"))
        if not m:
            continue
        f = [int(x) for x in m.group(1).split(",")]
        if f[0] < 0:
            continue
        k = tuple(f[:15])
        out[k] = (f[15], f[16], (m.group(2) or "").lstrip("/ ").strip())
        order.append(k)
    return out, order


def main():
    new_path = sys.argv[1]
    only = None
    for a in sys.argv[2:]:
        if a.startswith("--only-tiles"):
            only = {int(t) for t in a.split("=", 1)[1].split(",")}
    new_only = "--new-only" in sys.argv
    cur, order = parse(INC)
    new, norder = parse(new_path)
    head = [ln for ln in open(INC) if ln.startswith("//")]
    changed = added = 0
    for k in norder:
        tile, split, note = new[k]
        if k in cur:
            if new_only or cur[k][:2] == (tile, split) or (only and tile not in only):
                continue
            cur[k] = (tile, split, f"{note} (was tile {cur[k][0]} split {cur[k][1]})")
            changed += 1
        else:
            if only and not new_only:
                continue
            cur[k] = (tile, split, note)
            order.append(k)
            added += 1
    with open(INC, "w") as f:
        f.writelines(head)
        for k in order:
            tile, split, note = cur[k]
            f.write("    {" + ", ".join(map(str, k)) + f", {tile}, {split}}},  // {note}\n")
    print(f"{changed} replaced, {added} added, {len(order)} entries")


if __name__ == "__main__":
    main()
