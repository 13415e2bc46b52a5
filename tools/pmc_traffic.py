"""HBM traffic per launch of the fused kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

Reads ``<dir>/pmc_fetch/pmc_counter_collection.csv`` and ``<dir>/pmc_write/...`` (one pass each,
as tools/profile_round.sh collects them), keeps the dispatches of the kernel whose name contains
``--kernel``, and applies the gfx950 corrections of MI355X_MICROARCH.md (HBM / rocprofv3
section): counters are KiB; FETCH_SIZE reports half of the bytes of wide streaming reads, so it
is doubled; WRITE_SIZE is taken as is.  Writes the summary JSON (bench.py reads
``hbm_bytes_per_launch``).

    python tools/pmc_traffic.py gpurun_out/r01 --batch 512 -o profiles/r01/pmc_traffic.json
"""
import argparse
import csv
import json
import os


def per_dispatch(path, counter, kernel):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter or kernel not in row["Kernel_Name"]:
                continue
            d = row["Dispatch_Id"]
            vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])   # summed over XCD/agent rows
            name = row["Kernel_Name"]
    return vals, (name if vals else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="informer_forward_v4<64, false, 0, false, 1, false, false, 0>")
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--io-bytes-per-seq", type=int, default=7040)
    ap.add_argument("-o", "--out", required=True)
    args = ap.parse_args()
    fetch, name = per_dispatch(os.path.join(args.dir, "pmc_fetch", "pmc_counter_collection.csv"), "FETCH_SIZE",
                               args.kernel)
    write, _ = per_dispatch(os.path.join(args.dir, "pmc_write", "pmc_counter_collection.csv"), "WRITE_SIZE",
                            args.kernel)
    if not fetch or not write:
        raise SystemExit("no dispatches of the kernel in the PMC passes")
    f = sum(fetch.values()) / len(fetch)
    w = sum(write.values()) / len(write)
    total = int(round((2.0 * f + w) * 1024))
    res = {"kernel": name, "batch": args.batch, "fetch_size_kib_raw": round(f, 1), "write_size_kib": round(w, 1),
           "launches": [len(fetch), len(write)],
           "correction": "FETCH_SIZE x2 (gfx950 reports half of wide streaming reads), + WRITE_SIZE; KiB -> bytes",
           "hbm_bytes_per_launch": total, "algorithmic_io_bytes_per_launch": args.io_bytes_per_seq * args.batch}
    with open(args.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
