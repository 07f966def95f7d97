"""Short table of a rocprofv3 kernel_stats.csv: kernel (template args kept, parameters dropped),
calls, average and total ms, share of the GPU time.

    python tools/kstats.py <run_kernel_stats.csv> [top=25] [per_calls_divisor]
"""
import csv
import sys


def short(name):
    i = name.find("(")
    return name[:i] if i > 0 else name


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    div = float(sys.argv[3]) if len(sys.argv) > 3 else 0
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("%-70s %6s %9s %9s %6s" % ("kernel", "calls", "avg_ms", "total_ms", "pct"))
    for r in rows[:top]:
        t = float(r["TotalDurationNs"])
        extra = " %8.3f/step" % (t / 1e6 / div) if div else ""
        print("%-70s %6s %9.3f %9.2f %6.2f%s" % (short(r["Name"])[:70], r["Calls"],
                                                  float(r["AverageNs"]) / 1e6, t / 1e6,
                                                  100 * t / tot, extra))
    print("total GPU ms %.1f" % (tot / 1e6))


if __name__ == "__main__":
    main()
