"""Pipeline timeline report: host marks (BSHOT_HOST_TRACE csv) + rocprofv3 kernel trace.
usage: python pipeline_report.py host.csv kernel_trace.csv [frames]"""
import csv
import sys
from collections import defaultdict

host = [(n, int(t)) for n, t in csv.reader(open(sys.argv[1]))]
ker = []
for r in csv.DictReader(open(sys.argv[2])):
    ker.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]), r["Kernel_Name"].split("(")[0]))
ker.sort()
nshow = int(sys.argv[3]) if len(sys.argv) > 3 else 4
frames = [i for i, (n, _) in enumerate(host) if n == "M_frame"]
starts = [host[i][1] for i in frames]
print("frames", len(frames), "periods ms", [round((b - a) / 1e6, 3) for a, b in zip(starts, starts[1:])][-12:])
for fi in range(max(0, len(frames) - 1 - nshow), len(frames) - 1):
    t0, t1 = starts[fi], starts[fi + 1]
    ev = [(n, t) for n, t in host if t0 <= t < t1]
    print(f"--- frame {fi}: {(t1 - t0) / 1e6:.3f} ms")
    print("   host:", " ".join(f"{n}@{(t - t0) / 1e6:.2f}" for n, t in ev))
    busy = defaultdict(float)
    names = defaultdict(lambda: defaultdict(float))
    for s, e, st, nm in ker:
        a, b = max(s, t0), min(e, t1)
        if b > a:
            busy[st] += (b - a) / 1e6
            names[st][nm] += (b - a) / 1e6
    for st in sorted(busy):
        top = sorted(names[st].items(), key=lambda x: -x[1])[:5]
        print(f"   stream {st}: busy {busy[st]:.2f} ms  " + ", ".join(f"{k.split('::')[-1][:18]} {v:.2f}" for k, v in top))
    # per-stream first start / last end
    span = {}
    for s, e, st, nm in ker:
        if t0 <= s < t1:
            a = span.get(st, (s, e))
            span[st] = (min(a[0], s), max(a[1], e))
    print("   spans:", " ".join(f"s{st}:[{(a - t0) / 1e6:.2f},{(b - t0) / 1e6:.2f}]" for st, (a, b) in sorted(span.items())))

# whole-run summary: union of kernel intervals (any stream busy) vs wall time between the first
# and the last frame mark, and the busy time per stream
if len(starts) >= 2:
    t0, t1 = starts[0], starts[-1]
    iv = sorted((max(s, t0), min(e, t1)) for s, e, _, _ in ker if e > t0 and s < t1)
    union, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        union += cur_e - cur_s
    per = defaultdict(float)
    for s, e, st, nm in ker:
        a, b = max(s, t0), min(e, t1)
        if b > a:
            per[st] += (b - a) / 1e6
    nf = len(starts) - 1
    print(f"=== {nf} frames, {(t1 - t0) / 1e6 / nf:.3f} ms/frame; GPU busy (any stream) {union / 1e6 / nf:.3f} ms/frame "
          f"({union / (t1 - t0):.1%}); per stream ms/frame: " +
          " ".join(f"s{st}:{v / nf:.3f}" for st, v in sorted(per.items())))
