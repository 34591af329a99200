"""Per-kernel registers, spills, kernarg bytes and instruction counts of an ISA listing
(hipcc --offload-device-only -S):  python scripts/isa_stats.py file.s [name-filter]

Columns: kernarg segment bytes, SGPRs, SGPRs spilled (to VGPR lanes), VGPRs, VGPRs spilled, scratch bytes per
lane, instructions, f64 instructions, v_readlane / v_writelane (the SGPR spill traffic)."""
import re
import sys


def kernel_meta(s):
    """{kernel symbol: {metadata key: value}} from the listing's amdhsa.kernels block."""
    meta = {}
    blk = s[s.find("amdhsa.kernels:"):]
    for ent in re.split(r"\n  - ", blk)[1:]:
        m = re.search(r"\.name:\s+(\S+)", ent)
        if not m:
            continue
        meta[m.group(1)] = {k: int(v) for k, v in re.findall(r"\.(\w+):\s+(\d+)\s*$", ent, re.M)}
    return meta


def main():
    s = open(sys.argv[1]).read()
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    meta = kernel_meta(s)
    for m in re.finditer(r"^(_Z\w+):[^\n]*\n(.*?)\.Lfunc_end", s, re.S | re.M):
        name, body = m.group(1), m.group(2)
        if flt not in name or name not in meta:
            continue
        ins = [l for l in body.split("\n") if l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;")]
        f64 = sum(1 for l in ins if "_f64" in l)
        rl = sum(1 for l in ins if "v_readlane" in l)
        wl = sum(1 for l in ins if "v_writelane" in l)
        g = meta[name].get
        print("%-72s ka %4s sgpr %3s ssp %3s vgpr %3s vsp %3s scr %4s ins %5d f64 %5d rl/wl %d/%d"
              % (name[:72], g("kernarg_segment_size", "?"), g("sgpr_count", "?"), g("sgpr_spill_count", "?"),
                 g("vgpr_count", "?"), g("vgpr_spill_count", "?"), g("private_segment_fixed_size", "?"),
                 len(ins), f64, rl, wl))


if __name__ == "__main__":
    main()
