"""Per-launch HBM traffic of a kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_summary.py <fetch counter_collection.csv> <write counter_collection.csv> \
        <kernel substring> <out.json>

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE tallies 128-B requests of wide (16 B
per lane) coalesced reads at 64 B, i.e. reports exactly half of the bytes; WRITE_SIZE is exact
for 16-B-per-lane stores.  Both counters are in KiB.  traffic = 2 * FETCH + WRITE per launch.
"""
import csv
import json
import statistics
import sys


def per_launch(path, counter, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]]
    if not vals:
        raise SystemExit("no %s rows for kernel %r in %s" % (counter, kernel, path))
    return statistics.median(vals) * 1024.0, len(vals)


def main():
    fetch_csv, write_csv, kernel, out = sys.argv[1:5]
    fetch, nf = per_launch(fetch_csv, "FETCH_SIZE", kernel)
    write, nw = per_launch(write_csv, "WRITE_SIZE", kernel)
    res = {"kernel": kernel, "fetch_size_bytes_raw": fetch, "write_size_bytes": write,
           "fetch_bytes_corrected": 2.0 * fetch, "traffic_bytes": 2.0 * fetch + write,
           "launches": [nf, nw],
           "correction": "FETCH_SIZE x2 (gfx950 tallies 128-B requests at 64 B), WRITE_SIZE as is"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
