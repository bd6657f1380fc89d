"""profiles/r01_nce_fwdg_traffic.json from the FETCH_SIZE / WRITE_SIZE passes of
tools/nce_micro.py (rocprofv3 --pmc, separate passes; see tools/steps_final_r01.txt).

FETCH_SIZE is doubled (gfx950 reports half the bytes of 16-B/lane streaming reads,
MI355X_MICROARCH.md HBM section); WRITE_SIZE is taken as reported.
  python tools/make_traffic.py gpurun_out/pmcf gpurun_out/pmcw out.json [global_batch N D [nslots [kernel precision]]]"""
import csv
import glob
import json
import sys

KERNEL = sys.argv[8] if len(sys.argv) > 8 else "nce_grouped_fwdg_x3"  # default: x3_k and the pipelined x3p_k
PRECISION = sys.argv[9] if len(sys.argv) > 9 else "bf16x3"


def vals(d, counter):
    out = []
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
                out.append(float(r["Counter_Value"]))
    return out


def main():
    fetch = vals(sys.argv[1], "FETCH_SIZE")
    write = vals(sys.argv[2], "WRITE_SIZE")
    # tools/nce_micro.py --batch B shapes (bench batch 0): 4096 -> N 76850, D 16363
    batch, N, D = (int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])) if len(sys.argv) > 6 else (4096, 76850, 16363)
    ns = int(sys.argv[7]) if len(sys.argv) > 7 else 4  # partial slots per row (RSX_NCE_NSPLIT_FWD; 4 in rounds 1-3)
    f = sum(fetch) / len(fetch)
    w = sum(write) / len(write)
    hbm = int((2 * f + w) * 1024)
    # algorithmic: A and B rows (fp32) read once, the row-gradient partials [ns][N][128] written
    # once, the per-row (m, l, 0, 0) partials; images of B (hi/lo bf16) are written by the split
    # kernel outside this launch
    alg = 4 * (N + D) * 128 + ns * 4 * N * 128 + ns * 4 * 4 * N
    out = {
        "kernel": KERNEL + " (grouped LogQ forward fused with the row gradient, pipelined)",
        "precision": PRECISION, "global_batch": batch, "rows_N": N, "distinct_targets_D": D, "partial_slots": ns,
        "fetch_size_kb_raw": round(f, 1), "write_size_kb": round(w, 1),
        "hbm_bytes_per_launch": hbm,
        "correction": "FETCH_SIZE doubled (gfx950 reports half the bytes of 16-B/lane streaming reads, "
                      "MI355X_MICROARCH.md HBM section); WRITE_SIZE as reported",
        "algorithmic_bytes_per_launch": alg,
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over tools/nce_micro.py "
                  "--batch %d (bench batch 0 shapes)" % batch,
        "samples": {"fetch_kb": fetch, "write_kb": write},
    }
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("hbm_bytes_per_launch", "algorithmic_bytes_per_launch")}))


if __name__ == "__main__":
    main()
