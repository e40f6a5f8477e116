"""Per-kernel stats and one step's timeline (kernel starts/ends and gaps) from a
rocprofv3 --kernel-trace database (rocpd .db):
    python scripts/kt_timeline.py gpurun_out/<tag>/kt/run_results.db [anchor-substring]"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
anchor = sys.argv[2] if len(sys.argv) > 2 else "fast_kernel<true"
sfx = [r[0] for r in c.execute("select name from sqlite_master where type='table' and name like 'rocpd_kernel_dispatch%'")][0]
sfx = sfx.split("rocpd_kernel_dispatch_")[1]
names = {r[0]: r[1] for r in c.execute(f"select id, display_name from rocpd_info_kernel_symbol_{sfx}")}
rows = [(s, e, names.get(k, str(k))) for s, e, k in
        c.execute(f"select start, end, kernel_id from rocpd_kernel_dispatch_{sfx} order by start")]
st = collections.defaultdict(list)
for s, e, n in rows:
    st[n].append(e - s)
for n, d in sorted(st.items(), key=lambda kv: -sum(kv[1]))[:25]:
    print(f"{sum(d) / len(d) / 1e3:10.2f} us avg  x{len(d):4d}  {n[:110]}")
idx = [i for i, r in enumerate(rows) if anchor in r[2]]
if len(idx) >= 3:
    i0, i1 = idx[-2], idx[-1]
    print(f"\none step ({anchor} to the next): {(rows[i1][0] - rows[i0][0]) / 1e3:.1f} us")
    prev = None
    for s, e, n in rows[i0:i1 + 1]:
        gap = (s - prev) / 1e3 if prev else 0.0
        print(f"  +{gap:7.2f} gap  {(e - s) / 1e3:9.2f} us  {n[:90]}")
        prev = e
