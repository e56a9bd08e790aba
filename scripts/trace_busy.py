"""Steady-state device occupancy of a bench run from a rocprofv3 kernel trace.

usage: trace_busy.py <run_kernel_trace.csv>
The window is the longest run of sgr_res_kernel launches (one per frame) spaced < 6 ms apart, minus two frames at
each end; prints the ms per frame, the fraction of the window with at least one kernel running, the time share by
number of concurrent kernels, and each kernel's summed duration per frame (contended durations, not isolated ones).
"""
import csv, sys, collections
t=[x for x in csv.DictReader(open(sys.argv[1]))]
iv=sorted((int(x['Start_Timestamp']),int(x['End_Timestamp']),x['Kernel_Name']) for x in t)
sg=[s for s,e,n in iv if 'sgr_res_kernel' in n]
# longest run of consecutive sgr_res starts with gaps < 6 ms
best=(0,0,0); i=0
for j in range(1,len(sg)):
    if sg[j]-sg[j-1]>6e6: i=j
    if j-i>best[0]: best=(j-i,i,j)
n,i,j=best; a,b=sg[i+2],sg[j-2]
print('window frames', j-i-4, 'ms/frame %.3f'%((b-a)/1e6/(j-i-4)))
iv=[x for x in iv if a<=x[0]<b]
ev=[]
for s,e,_ in iv: ev.append((max(s,a),1)); ev.append((min(e,b),-1))
ev.sort(); cur=0; last=a; busy=0; hist=collections.Counter()
for tt,d in ev:
    if cur>0: busy+=tt-last
    hist[min(cur,6)]+=tt-last
    cur+=d; last=tt
span=b-a
print('busy %.1f%%'%(100*busy/span), {k:round(100*v/span,1) for k,v in sorted(hist.items())})
agg=collections.Counter()
for s,e,nm in iv: agg[nm.replace("(anonymous namespace)::","").replace("void ","").split("(")[0][:60]]+=e-s
fr=j-i-4
for k,v in agg.most_common(16): print('%-60s %7.3f ms/frame'%(k,v/1e6/fr))
