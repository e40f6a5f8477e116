"""One traced step of a kernel-trace CSV (rocprofv3 --kernel-trace --output-format csv):
every dispatch from one launch of the anchor kernel to the next, with start offset,
duration and the idle gaps between them.
    python scripts/step_timeline.py run_kernel_trace.csv --anchor 'fast_kernel<true' [--nth 6]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", required=True)
    ap.add_argument("--nth", type=int, default=6)
    a = ap.parse_args()
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                   for r in csv.DictReader(open(a.trace))), key=lambda x: x[0])
    idx = [i for i, r in enumerate(rows) if a.anchor in r[2]]
    i0, i1 = idx[a.nth - 1], idx[a.nth]
    t0 = rows[i0][0]
    prev_end = None
    busy = 0
    print(f"{'start_us':>9} {'dur_us':>8} {'gap_us':>7}  kernel")
    for s, e, n in rows[i0:i1 + 1]:
        gap = (s - prev_end) / 1000 if prev_end is not None else 0.0
        print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f} {gap:7.1f}  {n.replace('(anonymous namespace)::', '').split('(')[0][:90]}")
        if s < rows[i1][0]:
            busy += e - s
        prev_end = e
    period = (rows[i1][0] - t0) / 1000
    anchor = (rows[i0][1] - rows[i0][0]) / 1000
    print(f"step period {period:.1f} us: anchor kernel {anchor:.1f} us, other kernels "
          f"{busy / 1000 - anchor:.1f} us, idle {period - busy / 1000:.1f} us")


if __name__ == "__main__":
    main()
