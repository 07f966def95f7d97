"""Per-launch memory-side traffic of a kernel from rocprofv3 --pmc passes (one pass per CSV).

    python tools/pmc_summary.py <kernel substring> <out.json> <counter_collection.csv>...

Counters read (whichever the passes collected, median over the kernel's launches):
  FETCH_SIZE, WRITE_SIZE (KiB)   L2 -> fabric bytes.  gfx950 correction (MI355X_MICROARCH.md
                                 §HBM): FETCH_SIZE tallies the 128-B requests of wide (16 B per
                                 lane) coalesced reads at 64 B, i.e. reports half of the bytes;
                                 WRITE_SIZE is exact for 16-B-per-lane stores.
                                 traffic = 2 * FETCH + WRITE.
  TCC_HIT_sum, TCC_MISS_sum      L2 hit rate.
  TCC_EA0_RDREQ_DRAM_32B_sum     read requests the L2 sends toward DRAM, in 32-B units.
  TCC_EA0_WRREQ_DRAM_sum         write requests toward DRAM.
The memory-side counters include Infinity-Cache (MALL) hits: no gfx950 counter in
`rocprofv3 -L` separates them, so these bytes bound the HBM traffic from above (the compulsory
model in bench.py bounds it from below).
"""
import csv
import json
import statistics
import sys


def collect(paths, kernel):
    vals = {}
    for path in paths:
        for r in csv.DictReader(open(path)):
            if kernel in r["Kernel_Name"]:
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: (statistics.median(v), len(v)) for k, v in vals.items()}


def main():
    kernel, out = sys.argv[1:3]
    c = collect(sys.argv[3:], kernel)
    if not c:
        raise SystemExit("no counter rows for kernel %r" % kernel)
    res = {"kernel": kernel, "launches": {k: n for k, (_, n) in c.items()},
           "raw_median": {k: v for k, (v, _) in c.items()}}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        fetch, write = c["FETCH_SIZE"][0] * 1024.0, c["WRITE_SIZE"][0] * 1024.0
        res.update(fetch_size_bytes_raw=fetch, write_size_bytes=write,
                   fetch_bytes_corrected=2.0 * fetch, traffic_bytes=2.0 * fetch + write,
                   correction="FETCH_SIZE x2 (gfx950 tallies 128-B requests at 64 B), "
                              "WRITE_SIZE as is")
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        h, m = c["TCC_HIT_sum"][0], c["TCC_MISS_sum"][0]
        res["l2_hit_rate"] = h / (h + m) if h + m else None
    if "TCC_EA0_RDREQ_DRAM_32B_sum" in c:
        res["dram_side_read_bytes"] = 32.0 * c["TCC_EA0_RDREQ_DRAM_32B_sum"][0]
    res["note"] = ("memory-side counters include Infinity-Cache hits: an upper bound on HBM "
                   "bytes")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
