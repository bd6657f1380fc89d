"""Which kernels run concurrently with the loss kernels inside the training step, from a
rocprofv3 --kernel-trace of a step-only bench run: for every dispatch of the fused loss forward
and the column backward, the kernels of other queues whose interval overlaps it, with the
overlapped time; and the loss kernels' durations with and without any overlap.
  python tools/loss_overlap.py <rocprof out dir>"""
import collections
import csv
import glob
import sys

LOSS = ("nce_grouped_fwdg_x3", "nce_grouped_bwd_x3_k<false>")


def load(path):
    """(start, end, kernel name, queue) of every dispatch: kernel-trace CSVs or a rocpd database."""
    rows = []
    for f in glob.glob(path + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Queue_Id") or r.get("Stream_Id") or ""))
    for db in glob.glob(path + "/**/*.db", recursive=True) + ([path] if path.endswith(".db") else []):
        import sqlite3
        c = sqlite3.connect(db)
        tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
        kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
        ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
        for n, s, e, q in c.execute(f"select s.kernel_name, d.start, d.end, d.queue_id from {kd} d join {ks} s "
                                    f"on d.kernel_id = s.id"):
            rows.append((int(s), int(e), n, str(q)))
    rows.sort()
    return rows


def main():
    rows = load(sys.argv[1])
    for tag in LOSS:
        loss = [r for r in rows if tag in r[2]]
        over = collections.Counter()
        clean, hit = [], []
        for s, e, name, q in loss:
            ov = 0
            for s2, e2, n2, q2 in rows:
                if s2 >= e:
                    break
                if e2 <= s or (s2, e2, n2) == (s, e, name):
                    continue
                o = min(e, e2) - max(s, s2)
                if o > 0:
                    ov += o
                    over[n2.split("(")[0][:60]] += o
            (hit if ov else clean).append((e - s) / 1e6)
        print(f"== {tag}: {len(loss)} dispatches; {len(hit)} with overlap (avg "
              f"{sum(hit) / max(len(hit), 1):.3f} ms), {len(clean)} without (avg {sum(clean) / max(len(clean), 1):.3f} ms)")
        for n, t in over.most_common(12):
            print(f"   {t / 1e6 / max(len(loss), 1):8.3f} ms/dispatch  {n}")


if __name__ == "__main__":
    main()
