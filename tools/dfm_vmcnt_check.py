"""Checks the counted vmcnt waits of deepfm_rows2m_k in its ISA: at every field barrier B_g the
wave's own LDS-DMA of field g must be complete (no race) and, ideally, nothing younger waited for
(no over-wait). Reproduces the program's issue order of W1 / W2 DMAs (global_load_lds) and counts
every VMEM instruction (gathers, scratch) between them.

  hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include --offload-device-only -S \\
      llm-driven_content-based-feature_recommendation_system_amd/csrc/deepfm_fused.hip -o /tmp/dfm.s
  python tools/dfm_vmcnt_check.py /tmp/dfm.s 1      # MT = 1 (default shape), R = 3, F = 39
  python tools/dfm_vmcnt_check.py /tmp/dfm.s 2      # MT = 2"""
import re
import sys


def main():
    path, mt = sys.argv[1], int(sys.argv[2])
    F, R = 39, int(sys.argv[3]) if len(sys.argv) > 3 else 3
    nw = 8 // mt
    dp, idp = 16 // nw, 5 * mt
    name = "_ZN12_GLOBAL__N_115deepfm_rows2m_kILi39ELi%dELb1EEEvNS_5RArgsE" % mt
    s = open(path).read()
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    lines = [l.strip() for l in s[i:j].split("\n")]
    # program order of the LDS-DMAs: W2 pieces into unused blocks, fields 0..2, then per field the
    # W2 pieces of the id region (at field F-1-R), field f+3 after B_{f+1}, slot pieces after B_{F-1},
    # and the last two slots after layer 1
    tags = ["W2"] * (24 // nw) + ["F0"] * dp + ["F1"] * dp + ["F2"] * dp
    for f in range(F):
        if f == F - 1 - R:
            tags += ["W2"] * idp
        if f + 1 < F:
            if f + 3 < F:
                tags += ["F%d" % (f + 3)] * dp
            if f + 1 == F - 1:
                tags += ["W2"] * (2 * dp)
    tags += ["W2"] * (2 * dp)
    ops, complete, bar, k, races, over = [], 0, 0, 0, 0, []
    for l in lines:
        op = l.split(" ")[0]
        if op.startswith(("global_load", "global_store", "scratch_", "buffer_")):
            if op.startswith("global_load_lds"):
                ops.append(tags[k])
                k += 1
            else:
                ops.append(op)
        m = re.match(r"s_waitcnt\s+(.*)", l)
        if m and "vmcnt" in m.group(1):
            n = int(re.search(r"vmcnt\((\d+)\)", m.group(1)).group(1))
            complete = max(complete, len(ops) - n)
        if op == "s_barrier":
            if bar < F:
                idx = max(x for x, t in enumerate(ops) if t == "F%d" % bar)
                if idx >= complete:
                    print("B_%d: RACE (field %d's DMA not waited for)" % (bar, bar))
                    races += 1
                elif complete != idx + 1:
                    over.append((bar, complete - idx - 1))
            bar += 1
    print("LDS-DMA instructions %d of %d expected, barriers %d, races %d, over-waits %s" % (k, len(tags), bar, races, over))
    sys.exit(1 if races or k != len(tags) else 0)


if __name__ == "__main__":
    main()
