"""Idle time inside the training step from a rocprofv3 --kernel-trace of a step-only bench run:
per step (fused-loss-forward dispatch to the next), the union of kernel intervals over all
streams, the idle remainder and the largest gaps with the kernels either side.
  python tools/step_gaps.py <rocprof out dir> [n_steps]"""
import collections
import csv
import glob
import sys

MARK = "nce_grouped_fwdg_x3"


def main():
    sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
    from loss_overlap import load
    rows = [(s, e, n[:70]) for s, e, n, _ in load(sys.argv[1])]
    marks = [i for i, r in enumerate(rows) if MARK in r[2]]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    gaps = collections.Counter()
    tot_p = tot_b = 0
    for a, b in zip(marks[-n - 1:-1], marks[-n:]):
        seg = rows[a:b]
        t0, t1 = seg[0][0], rows[b][0]
        busy, cur_s, cur_e, prev = 0, seg[0][0], seg[0][1], seg[0][2]
        for s, e, name in seg[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                gaps[(prev, name)] += s - cur_e
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            prev = name
        busy += cur_e - cur_s
        tot_p += t1 - t0
        tot_b += busy
        print(f"step {(t1 - t0) / 1e6:7.3f} ms  busy {busy / 1e6:7.3f}  idle {(t1 - t0 - busy) / 1e6:6.3f}  "
              f"dispatches {b - a}")
    k = len(marks[-n:])
    print(f"mean step {tot_p / k / 1e6:.3f} ms, busy {tot_b / k / 1e6:.3f}, idle {(tot_p - tot_b) / k / 1e6:.3f}")
    for (p, q), g in gaps.most_common(25):
        print(f"{g / k / 1e3:8.1f} us/step  {p}  ->  {q}")


if __name__ == "__main__":
    main()
