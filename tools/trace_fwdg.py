"""profiles/rNN_bench_nce_fwdg_from_trace.json from a rocprofv3 --kernel-trace of bench.py:
the fused LogQ forward's dispatch durations in launch order (warm-up + timed steps of the
headline line first), their timed-step average and the kernel-only roofline fraction.
  python tools/trace_fwdg.py <rocprof out dir> <bench json under rocprof> <out.json>"""
import csv
import glob
import json
import re
import sys

KERNEL = "nce_grouped_fwdg_x3"
PEAK = 2516.8 / 3  # bf16x3 TF (bench.py)


def main():
    rows = []
    for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    b = json.loads(open(sys.argv[2]).read().strip().split("\n")[-1])
    warm, steps = b["warmup"], b["steps"]
    ms = [round((e - s) / 1e6, 4) for s, e, _ in rows]
    head = ms[:warm + steps]
    timed = head[warm:]
    flops = b["roofline"]["flops_per_launch"]
    avg = sum(timed) / len(timed)
    out = {"source": "rocprofv3 --kernel-trace --stats -- python bench.py (same invocation as the bench line)",
           "kernel": re.search(r"nce_grouped_fwdg_\w+", rows[0][2]).group(0) if rows else KERNEL,
           "headline_dispatches_in_order_ms": head, "warmup": warm, "steps": steps,
           "timed_avg_kernel_ms": round(avg, 4),
           "bench_roofline_avg_launch_ms_same_run": b["roofline"]["avg_launch_ms"],
           "note": "the bench's HIP-event window is the op (B split + fused kernel + merge + reduce); later "
                   "dispatches belong to the secondary lines",
           "flops_per_launch": flops, "kernel_only_frac": round(flops / (avg * 1e-3) / 1e12 / PEAK, 4)}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
