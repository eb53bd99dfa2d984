"""The last complete V-cycle of a rocprofv3 kernel trace (between the last two k_sumsq_finish launches),
kernel time per (name, grid) and the wall span:   python tools/vc_breakdown.py <kernel_trace.csv> [top]"""
import csv, collections, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
names=[r['Kernel_Name'].replace('(anonymous namespace)::','').split('(')[0] for r in rows]
t0=[int(r['Start_Timestamp']) for r in rows]; t1=[int(r['End_Timestamp']) for r in rows]
fin=[i for i,n in enumerate(names) if 'sumsq_finish' in n]
a,b=fin[-2]+1, fin[-1]
agg=collections.defaultdict(lambda:[0,0.0])
for i in range(a,b+1):
    g=int(rows[i]['Grid_Size_X'])*int(rows[i]['Grid_Size_Y'])*int(rows[i]['Grid_Size_Z'])
    key=(names[i][:44], g)
    agg[key][0]+=1; agg[key][1]+=(t1[i]-t0[i])/1e3
tot=sum(v[1] for v in agg.values())
print('kernel time sum (us):', round(tot,1), ' wall (us):', round((t1[b]-t0[a])/1e3,1), 'launches', b-a+1)
for k,v in sorted(agg.items(), key=lambda kv:-kv[1][1])[:int(sys.argv[2]) if len(sys.argv)>2 else 20]: print(f"{k[0]:46s} grid={k[1]:>10d} n={v[0]:3d} {v[1]:9.1f} us")
if len(sys.argv) > 3 and sys.argv[3] == "--seq":
    # every launch of that cycle in order: duration and the idle gap since the previous launch ended
    print("\nlaunch sequence (us): duration, gap before")
    for i in range(a, b + 1):
        g = int(rows[i]['Grid_Size_X']) * int(rows[i]['Grid_Size_Y']) * int(rows[i]['Grid_Size_Z'])
        gap = (t0[i] - t1[i - 1]) / 1e3 if i > a else 0.0
        print(f"  {names[i][:50]:52s} grid={g:>9d} {(t1[i]-t0[i])/1e3:8.1f} {gap:6.1f}")
