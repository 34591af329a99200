"""Per-kernel VGPRs, scratch bytes and instruction count of an ISA listing
(hipcc --offload-device-only -S):  python scripts/isa_stats.py file.s [name-filter]"""
import re
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
meta = {}
for m in re.finditer(r"\.name:\s+(\S+)\n(.*?)(?=\n  - |\n\.\.\.)", s, re.S):
    body = m.group(2)
    g = lambda k: (re.search(r"\.%s:\s+(\d+)" % k, body) or [None, "?"])[1]
    meta[m.group(1)] = (g("vgpr_count"), g("private_segment_fixed_size"))
for m in re.finditer(r"^(_Z\w+):[^\n]*\n(.*?)\.Lfunc_end", s, re.S | re.M):
    name, body = m.group(1), m.group(2)
    if flt not in name:
        continue
    ins = [l for l in body.split("\n") if l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;")]
    f64 = sum(1 for l in ins if "_f64" in l)
    v, sc = meta.get(name, ("?", "?"))
    print("%-70s vgpr %4s scratch %5s  instrs %6d  f64 %5d" % (name[:70], v, sc, len(ins), f64))
