"""Pipeline timeline of a bench run: rocprofv3 kernel/copy trace (csv) + BSHOT_HOST_TRACE marks on the
same steady clock. Prints the GPU busy fraction (union of all streams), kernel time per stream, the
main stream's kernel vs gap time, and one steady-state sweep: main-thread marks with the main-stream
operations, then the start times of the other streams' kernels.
usage: python pipeline_timeline.py <trace dir (…_kernel_trace.csv, …_memory_copy_trace.csv)> <host.csv>"""
import collections
import csv
import glob
import sys

d, hfile = sys.argv[1], sys.argv[2]
kt = glob.glob(d + "/*kernel_trace.csv")[0]
ct = glob.glob(d + "/*memory_copy_trace.csv")
K = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]),
      r["Kernel_Name"].split("(")[0].replace("bsk::", "").replace("void rocprim::ROCPRIM_400200_NS::detail::", "rocprim:")[:30])
     for r in csv.DictReader(open(kt))]
if ct:
    K += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]), "copy " + r["Direction"][:4])
          for r in csv.DictReader(open(ct[0]))]
K.sort()
t0 = K[int(len(K) * 0.4)][0]
t1 = K[-1][1]
W = [k for k in K if k[0] >= t0]
ev = sorted([(s, 1) for s, e, *_ in W] + [(e, -1) for s, e, *_ in W])
busy, cur, last = 0, 0, t0
for t, dd in ev:
    if cur > 0:
        busy += t - last
    cur += dd
    last = t
print(f"window {(t1 - t0) / 1e6:.1f} ms (last 60% of the trace), GPU busy (any stream) {busy / (t1 - t0):.3f}")
H = [(n, int(t)) for n, t in csv.reader(open(hfile))]
fr = [t for n, t in H if n == "M_frame"]
nsw = sum(1 for t in fr if t0 <= t < t1)
by = collections.defaultdict(lambda: [0, collections.Counter()])
for s, e, st, n in W:
    by[st][0] += e - s
    by[st][1][n] += e - s
for st, (tot, names) in sorted(by.items()):
    top = ", ".join(f"{n} {v / 1e3 / max(1, nsw):.0f}" for n, v in names.most_common(6))
    print(f"stream {st}: {tot / 1e3 / max(1, nsw):.0f} us kernel time per sweep; top (us/sweep): {top}")
main = [k for k in W if "ham_min" in k[3]][0][2]
M = [k for k in W if k[2] == main]
gaps = sum(max(0, b[0] - a[1]) for a, b in zip(M, M[1:]))
print(f"main stream {main}: kernels {sum(e - s for s, e, *_ in M) / 1e3 / max(1, nsw):.0f} us, gaps {gaps / 1e3 / max(1, nsw):.0f} us per sweep")
i = len(fr) // 2 + 3
a, b = fr[i], fr[i + 1]
print(f"\none sweep: period {(b - a) / 1e3:.0f} us (times in us from M_frame)")
rows = [(t, "host", n) for n, t in H if a <= t < b]
rows += [(s, f"s{st}", f"{n} [{(e - s) / 1e3:.1f}]") for s, e, st, n in K if e >= a and s < b]
rows.sort()
for t, k, n in rows:
    if k in ("host", f"s{main}"):
        print(f"{(t - a) / 1e3:8.1f} {k:5s} {n}")
for st in sorted(by):
    if st != main:
        print(f"stream {st}: " + " ".join(f"{(t - a) / 1e3:.0f}:{n}" for t, k, n in rows if k == f"s{st}" and "rocprim" not in n))
