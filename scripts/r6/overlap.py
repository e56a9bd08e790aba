"""Which kernels run beside the slow launches of one kernel (a rocprofv3 kernel trace CSV): overlap time per other
kernel as a fraction of the slow launches' total time.  usage: overlap.py trace.csv [kernel-substring] [slow_us]"""
import collections, csv, re, sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", n)[:48]


rows = list(csv.DictReader(open(sys.argv[1])))
target = sys.argv[2] if len(sys.argv) > 2 else "sod_step_kernel"
slow_us = float(sys.argv[3]) if len(sys.argv) > 3 else 30.0
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"]) for r in rows)
for label, cond in (("slow", lambda d: d > slow_us * 1e3), ("fast", lambda d: d < 12e3)):
    acc, n, tot = collections.Counter(), 0, 0
    for i, (s, e, nm, q) in enumerate(ks):
        if target not in nm or not cond(e - s):
            continue
        n, tot = n + 1, tot + e - s
        for s2, e2, nm2, q2 in ks:
            if s2 >= e:
                break
            if e2 <= s or (s2 == s and nm2 == nm):
                continue
            acc[nm2] += min(e, e2) - max(s, s2)
    print(label, n, "avg %.1f us" % (tot / max(n, 1) / 1e3))
    for k, t in acc.most_common(10):
        print("   %-48s %.2f" % (k, t / max(tot, 1)))
