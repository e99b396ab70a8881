"""Per-queue busy fractions over the timed region of a rocprofv3 kernel trace of the bench
(tools/gpu_steps.sh prof): the window is the span of the last K chain_adpcm launches (one per
engine block: K = 40 for the paired 20-step C3 run), from the first of them to the last one's end.

usage: python3 tools/queue_busy.py <kernel_trace.csv> [K]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    enc = [r for r in rows if "chain_adpcm" in r["Kernel_Name"]][-k:]
    t0, t1 = int(enc[0]["Start_Timestamp"]), int(enc[-1]["End_Timestamp"])
    busy = collections.defaultdict(list)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        s, e = max(int(r["Start_Timestamp"]), t0), min(int(r["End_Timestamp"]), t1)
        if e <= s:
            continue
        q = r["Queue_Id"]
        busy[q].append((s, e))
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("owrx::", "")
        per[q][name[:34]] += (e - s) / 1e6
    print("window: the last %d chain_adpcm launches, %.3f ms" % (k, (t1 - t0) / 1e6))
    for q in sorted(busy, key=lambda q: -sum(e - s for s, e in busy[q])):
        iv = sorted(busy[q])
        tot, cs, ce = 0, None, None
        for s, e in iv:  # union of intervals
            if cs is None or s > ce:
                if cs is not None:
                    tot += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        tot += ce - cs
        top = sorted(per[q].items(), key=lambda x: -x[1])[:5]
        print("queue %s: busy %5.1f %%  %s" % (q, 100.0 * tot / (t1 - t0),
                                             ", ".join("%s %.2f ms" % (n, v) for n, v in top)))


if __name__ == "__main__":
    main()
