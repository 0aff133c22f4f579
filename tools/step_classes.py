"""Per-kernel-class totals of ONE training step (adam_fused to adam_fused) in a rocprofv3 kernel trace.
usage: python tools/step_classes.py <run_kernel_trace.csv> [rows]"""
import csv,re,sys
from collections import Counter
rows=sorted(csv.DictReader(open(sys.argv[1])), key=lambda r:int(r['Start_Timestamp']))
idx=[i for i,r in enumerate(rows) if 'adam_fused' in r['Kernel_Name']]
a,b=idx[-3],idx[-2]
step=rows[a+1:b+1]
c=Counter(); n=Counter()
for r in step:
    k=r['Kernel_Name'].replace('void ','').replace('(anonymous namespace)::','')
    k=re.sub(r'\(.*','',k)[:75]
    c[k]+=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3; n[k]+=1
t0=int(step[0]['Start_Timestamp']); t1=int(step[-1]['End_Timestamp'])
print('kernels',len(step),'busy',round(sum(c.values()),1),'span',round((t1-t0)/1e3,1))
for k,v in c.most_common(int(sys.argv[2]) if len(sys.argv)>2 else 30): print(f"{v:8.1f} {n[k]:4d} {v/n[k]:7.1f} {k}")
