"""Per-kernel totals of a rocprofv3 kernel trace (sqlite): trace_agg.py DIR [TOP]"""
import sqlite3,glob,collections,re,sys
db=glob.glob(sys.argv[1]+'/**/*.db',recursive=True)[0]
c=sqlite3.connect(db)
tabs=[r[0] for r in c.execute("select name from sqlite_master where type='table'")]
ks=[t for t in tabs if t.startswith('rocpd_info_kernel_symbol')][0]
kd=[t for t in tabs if t.startswith('rocpd_kernel_dispatch')][0]
rows=list(c.execute(f"select s.display_name, d.start, d.end, d.grid_size_x, d.workgroup_size_x from {kd} d join {ks} s on d.kernel_id=s.id order by d.start"))
def short(n):
    n=n.replace('(anonymous namespace)::','').replace('void ','')
    n=re.sub(r'\(.*','',n); return n[:90]
agg=collections.defaultdict(lambda:[0,0.0])
for n,s,e,g,w in rows:
    a=agg[short(n)]; a[0]+=1; a[1]+=(e-s)/1e6
tot=sum(a[1] for a in agg.values())
print('total kernels',len(rows),'ms',round(tot,2), 'wall', (rows[-1][2]-rows[0][1])/1e6)
for k,(cnt,ms) in sorted(agg.items(),key=lambda x:-x[1][1])[:int(sys.argv[2]) if len(sys.argv)>2 else 70]:
    print(f'{ms:9.3f} {cnt:6d} {k}')
