"""Timeline summary of a host-pipeline trace (rocprofv3 --kernel-trace --memory-copy-trace csv):
per job (events separated by more than GAP_US of idle, default 300), the busy time and bytes of each copy direction,
the kernels, the idle gaps inside each direction's stream of copies, and the job's span.
usage: python tools/copy_trace.py DIR/PREFIX [GAP_US]  (reads PREFIX_memory_copy_trace.csv and
PREFIX_kernel_trace.csv)"""
import csv
import json
import sys


def rows(path):
    try:
        with open(path) as f:
            return list(csv.DictReader(f))
    except FileNotFoundError:
        return []


def main(prefix: str, gap_us: float = 300.0) -> None:
    ev = []
    for r in rows(prefix + "_memory_copy_trace.csv"):
        d = "h2d" if "HOST_TO_DEVICE" in r["Direction"] else "d2h" if "DEVICE_TO_HOST" in r["Direction"] else "other"
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), d, r.get("Stream_Id")))
    for r in rows(prefix + "_kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kernel", r.get("Stream_Id")))
    ev.sort()
    jobs, cur, last_end = [], [], None
    for e in ev:
        if last_end is not None and e[0] - last_end > gap_us * 1e3:
            jobs.append(cur)
            cur = []
        cur.append(e)
        last_end = e[1] if last_end is None else max(last_end, e[1])
    if cur:
        jobs.append(cur)
    for k, job in enumerate(jobs):
        t0 = min(e[0] for e in job)
        t1 = max(e[1] for e in job)
        out = {"job": k, "span_us": round((t1 - t0) / 1e3, 1), "events": len(job)}
        for kind in ("h2d", "d2h", "kernel"):
            sel = sorted((e for e in job if e[2] == kind), key=lambda e: e[0])
            if not sel:
                continue
            busy = sum(e[1] - e[0] for e in sel)
            gaps = [max(0, b[0] - a[1]) for a, b in zip(sel, sel[1:])]
            out[kind] = {"n": len(sel), "busy_us": round(busy / 1e3, 1),
                         "first_start_us": round((sel[0][0] - t0) / 1e3, 1),
                         "last_end_us": round((sel[-1][1] - t0) / 1e3, 1),
                         "gaps_us": round(sum(gaps) / 1e3, 1),
                         "max_gap_us": round(max(gaps, default=0) / 1e3, 1),
                         "streams": sorted({e[3] for e in sel})}
        print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 300.0)
