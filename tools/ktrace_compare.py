"""Per-kernel comparison of two rocprofv3 --kernel-trace CSVs of ``bench/profile_model.py``: sums each kernel's
dispatches from the last stem launch on (the second, timed forward).

    python tools/ktrace_compare.py before/run_kernel_trace.csv after/run_kernel_trace.csv
"""
import csv,sys,collections
def load(path):
    rows=list(csv.DictReader(open(path)))
    rows.sort(key=lambda r:int(r['Start_Timestamp']))
    idx=[i for i,r in enumerate(rows) if 'stem_pool_direct' in r['Kernel_Name']]
    rows=rows[idx[-1]:]
    agg=collections.OrderedDict()
    for r in rows:
        n=r['Kernel_Name'].replace('void ','').replace('(anonymous namespace)::','').split('(')[0][:70]
        d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3
        a=agg.setdefault(n,[0,0.0]); a[0]+=1; a[1]+=d
    return agg
a=load(sys.argv[1]); b=load(sys.argv[2])
keys=list(dict.fromkeys(list(a)+list(b)))
ta=tb=0
for k in sorted(keys,key=lambda k:-max(a.get(k,[0,0])[1],b.get(k,[0,0])[1])):
    x=a.get(k,[0,0]); y=b.get(k,[0,0]); ta+=x[1]; tb+=y[1]
    print(f"{x[1]:8.1f} ({x[0]:2}) {y[1]:8.1f} ({y[0]:2})  {k}")
print(f"total {ta:.1f} {tb:.1f}")
