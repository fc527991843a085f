#!/usr/bin/env python3
"""Per-kernel instruction mix of a gfx950 assembly file (hipcc -save-temps output).

    python tools/isa_stats.py k-hip-amdgcn-amd-amdhsa-gfx950.s [substring ...] [--top N]

Prints, for every kernel whose mangled name contains one of the substrings: static VALU
count, v_mov count, exec-mask branches, readfirstlane (waterfall loops), VGPRs, scratch.
"""
import re
import sys


def kernels(path):
    cur, body, meta = None, [], {}
    with open(path) as f:
        lines = f.read().splitlines()
    out = {}
    for ln in lines:
        m = re.match(r"^(_Z[A-Za-z0-9_]+):\s*(;.*)?$", ln)
        if m:
            cur, body = m.group(1), []
            out[cur] = body
            continue
        if cur is not None:
            if ln.startswith(".Lfunc_end"):
                cur = None
                continue
            body.append(ln)
    # metadata: .name / .vgpr_count / .private_segment_fixed_size
    name = None
    for ln in lines:
        m = re.match(r"^\s+\.name:\s+(\S+)", ln)
        if m:
            name = m.group(1)
            meta.setdefault(name, {})
        m = re.match(r"^\s+\.(vgpr_count|sgpr_count|private_segment_fixed_size|group_segment_fixed_size):\s+(\d+)", ln)
        if m and name:
            meta[name][m.group(1)] = int(m.group(2))
    return out, meta


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    top = 0
    if "--top" in sys.argv:
        top = int(sys.argv[sys.argv.index("--top") + 1])
        args = [a for a in args if a != str(top)]
    path, subs = args[0], args[1:]
    ks, meta = kernels(path)
    for k, body in ks.items():
        if subs and not any(s in k for s in subs):
            continue
        ins = [re.match(r"^\s+([a-z_0-9]+)", l) for l in body]
        ops = [m.group(1) for m in ins if m]
        valu = sum(1 for o in ops if o.startswith("v_"))
        md = meta.get(k, {})
        print("%-90s VALU %5d mov %4d br %3d rfl %3d vgpr %s scratch %s" % (
            k[:90], valu, sum(o == "v_mov_b32_e32" for o in ops), sum(o.startswith("s_and_saveexec") for o in ops),
            sum(o == "v_readfirstlane_b32" for o in ops), md.get("vgpr_count"), md.get("private_segment_fixed_size")))
        if top:
            from collections import Counter
            for o, n in Counter(ops).most_common(top):
                print("      %5d %s" % (n, o))


if __name__ == "__main__":
    main()
