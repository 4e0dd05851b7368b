"""Per-kernel wait/load census of a hipcc -save-temps assembly file: s_waitcnt vmcnt(0) count,
counted vmcnt waits, vector global loads (not LDS-DMA), scalar loads and instruction count, to
spot epilogues or loops that drain the whole vector-memory queue.
Usage: python tools/isa_waits.py file.s [name filter]"""
import re
import subprocess
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"\n([_A-Za-z0-9]+):[^\n]*\n", s):
    name = m.group(1)
    if not name.startswith("_Z") or flt not in name:
        continue
    end = s.find(".Lfunc_end", m.start())
    if end < 0:
        continue
    lines = [l.strip() for l in s[m.start():end].split("\n") if l.startswith("\t")]
    if not lines:
        continue
    vm0 = sum("s_waitcnt vmcnt(0)" in l for l in lines)
    vmn = sum("s_waitcnt vmcnt(" in l for l in lines) - vm0
    gl = sum(l.startswith(("global_load", "buffer_load")) and " lds" not in l for l in lines)
    sl = sum(l.startswith("s_load") for l in lines)
    dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    print(f"{dm[:90]:90s} vmcnt0 {vm0:4d} vmcntN {vmn:4d} vload {gl:4d} sload {sl:3d} n {len(lines)}")
