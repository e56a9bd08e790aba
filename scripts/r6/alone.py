"""Time each kernel runs alone on the device (no other kernel in flight) and beside others, per frame, over the main
run of a bench kernel trace (the span in which every frame slot's stream runs self-guided searches), and the time share
by number of kernels in flight.  usage: alone.py run_kernel_trace.csv"""
import collections, csv, re, sys
t = list(csv.DictReader(open(sys.argv[1])))
short = lambda n: re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "").replace("void ", ""))[:44]
iv = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), short(x["Kernel_Name"])) for x in t)
# the main run: the span of the self-guided searches of every stream but the busiest one's tail -- a bench trace ends
# with slot 0 alone (the roofline's isolated phase), which a window of consecutive launches would pick instead
streams = collections.defaultdict(list)
for x in t:
    if "sgr_res_kernel" in x["Kernel_Name"]: streams[x["Stream_Id"]].append(int(x["Start_Timestamp"]))
others = sorted(k for k in streams if len(streams) == 1 or k != max(streams, key=lambda q: len(streams[q])))
if len(streams) > 1:
    lo = max(min(streams[k]) for k in others)
    hi = min(max(streams[k]) for k in others)
    sg = sorted(v for k in streams for v in streams[k] if lo <= v <= hi)
else:
    sg = sorted(streams[others[0]])
a, b = sg[2], sg[-3]
nf = len([v for v in sg if a <= v < b])
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
hist = collections.Counter()
run2 = collections.Counter(); last = a
for tm, d, nm in ev:
    hist[min(6, sum(1 for c in run2.values() if c > 0))] += tm - last
    run2[nm] += d; last = tm
tot = sum(hist.values())
print("frames", nf, "ms/frame %.3f" % ((b - a) / 1e6 / nf), "kernels in flight (% of time):",
      {k: round(100.0 * v / tot, 1) for k, v in sorted(hist.items())})
for k, v in alone.most_common(16):
    print("  %-44s alone %7.1f us/frame   in flight %7.1f us/frame" % (k, v / 1e3 / nf, beside[k] / 1e3 / nf))
