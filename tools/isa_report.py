"""Summarise a hipcc -S gfx950 assembly file: per kernel VGPR/SGPR/spills and
instruction mix.  Usage: python tools/isa_report.py file.s [name-filter]"""
import re
import sys
from collections import Counter


def main(path, filt=""):
    s = open(path).read()
    meta = {}
    for ent in re.split(r"\n\s+- \.agpr_count:", s.split("amdhsa.kernels:")[-1])[1:]:
        g = lambda k: (re.search(r"\.%s:\s+(\S+)" % k, ent) or [None, "?"])[1]
        meta[g("name")] = dict(vgpr=g("vgpr_count"), sgpr=g("sgpr_count"),
                               vspill=g("vgpr_spill_count"), sspill=g("sgpr_spill_count"),
                               scratch=g("private_segment_fixed_size"), lds=g("group_segment_fixed_size"))
    for m in re.finditer(r"\n(_Z\w+):[^\n]*\n(.*?)\n\.Lfunc_end", s, re.S):
        name, body = m.group(1), m.group(2)
        if filt and filt not in name:
            continue
        ins = [l.split()[0] for l in body.splitlines()
               if l.startswith("\t") and not l.startswith("\t.") and not l.strip().startswith(";")]
        c = Counter(ins)
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        print(f"{name[-60:]}: n={len(ins)} valu={valu} {meta.get(name, {})}")
        print("   ", ", ".join(f"{k}:{v}" for k, v in c.most_common(18)))


if __name__ == "__main__":
    main(*sys.argv[1:])
