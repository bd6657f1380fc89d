"""HBM bytes of one rsx_tower_fwd / rsx_tower_bwd call from rocprofv3 --pmc passes over
tools/tower_micro.py (FETCH_SIZE and WRITE_SIZE in separate runs): the dispatches between the micro's
marker kernels (torch.cuda._sleep) are attributed to the forward or the backward call; torch's own
kernels in the backward window (autograd's gradient fills) are left out. FETCH_SIZE is doubled
(MI355X_MICROARCH.md: gfx950 reports half the bytes of 16-B/lane streaming reads), WRITE_SIZE as
reported; the first two iterations (warm-up) are dropped.

  python tools/tower_traffic.py gpurun_out/pmcf gpurun_out/pmcw out.json [T R U]
"""
import csv
import glob
import json
import sys


def phases(d, counter):
    rows = []
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    out, cur, phase, marks = {"fwd": [], "bwd": []}, 0.0, None, 0
    for _, name, v in rows:
        if "sleep" in name.lower() or "spin" in name.lower():
            if phase is not None:
                out[phase].append(cur)
            marks += 1
            phase = ("fwd", "bwd", None)[(marks - 1) % 3]
            cur = 0.0
            continue
        if phase is None or name.startswith("void at::") or name.startswith("at::") or "rocprim" in name:
            continue
        cur += v
    return {k: v[2:] for k, v in out.items()}


def main():
    f = phases(sys.argv[1], "FETCH_SIZE")
    w = phases(sys.argv[2], "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over tools/tower_micro.py "
                     "(headline batch 8192, both views, tail rows, dropout 0.2)",
           "correction": "FETCH_SIZE doubled (MI355X_MICROARCH.md HBM section); WRITE_SIZE as reported; KB -> bytes"}
    if len(sys.argv) > 6:
        res.update({"packed_tokens_T": int(sys.argv[4]), "tail_rows_R": int(sys.argv[5]), "user_rows_U": int(sys.argv[6])})
    for ph, name in (("fwd", "tower_fwd"), ("bwd", "tower_bwd")):
        fk = sum(f[ph]) / max(len(f[ph]), 1)
        wk = sum(w[ph]) / max(len(w[ph]), 1)
        res[name] = {"fetch_kb_raw": round(fk, 1), "write_kb": round(wk, 1),
                     "hbm_bytes_per_call": int((2 * fk + wk) * 1024), "calls": len(f[ph])}
    json.dump(res, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
