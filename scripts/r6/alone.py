"""Time each kernel runs alone on the device (no other kernel in flight) and beside others, per frame, over the steady
window of a bench kernel trace (as trace_busy.py).  usage: alone.py run_kernel_trace.csv"""
import collections, csv, re, sys
t = list(csv.DictReader(open(sys.argv[1])))
short = lambda n: re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "").replace("void ", ""))[:44]
iv = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), short(x["Kernel_Name"])) for x in t)
sg = [s for s, e, n in iv if "sgr_res_kernel" in n]
best, i = (0, 0, 0), 0
for j in range(1, len(sg)):
    if sg[j] - sg[j - 1] > 6e6: i = j
    if j - i > best[0]: best = (j - i, i, j)
n, i, j = best
a, b = sg[i + 2], sg[j - 2]
nf = j - i - 4
ev = []
for s, e, nm in iv:
    if e <= a or s >= b: continue
    ev.append((max(s, a), 1, nm)); ev.append((min(e, b), -1, nm))
ev.sort()
run = collections.Counter(); alone = collections.Counter(); beside = collections.Counter(); last = a
for tm, d, nm in ev:
    live = [k for k, c in run.items() if c > 0]
    if len(live) == 1: alone[live[0]] += tm - last
    for k in live: beside[k] += tm - last
    run[nm] += d; last = tm
print("frames", nf, "ms/frame %.3f" % ((b - a) / 1e6 / nf))
for k, v in alone.most_common(16):
    print("  %-44s alone %7.1f us/frame   in flight %7.1f us/frame" % (k, v / 1e3 / nf, beside[k] / 1e3 / nf))
