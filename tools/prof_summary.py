#!/usr/bin/env python3
"""Summarise rocprofv3 --kernel-trace --stats output into markdown (for profiles/).

Accepts the CSV stats file (``--output-format csv``: *_kernel_stats.csv), the default rocpd
SQLite database (*_results.db; per-kernel totals plus VGPR/LDS use), or the kernel-trace CSV
(*_kernel_trace.csv: serving dispatches only, engine start-up excluded)."""
import csv
import sqlite3
import sys


def _rows_csv(path):
    for r in csv.DictReader(open(path)):
        yield (r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), None, None)


def _rows_db(path):
    c = sqlite3.connect(path)
    q = ("select name, count(*), sum(duration), max(vgpr_count + accum_vgpr_count), "
         "max(lds_size) from kernels group by name order by sum(duration) desc")
    yield from c.execute(q)


def _rows_trace_serving(path):
    """Per-kernel totals from a --kernel-trace CSV (*_kernel_trace.csv), counting only the
    dispatches from the first prefill-attention kernel on: the engine's start-up work (GEMM
    tuning candidates, hipGraph capture warm-ups, the KV-cache zero fill) runs before any
    request is served, and none of it is serving time."""
    rows = list(csv.DictReader(open(path)))
    key = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
    t0 = min((int(r["Start_Timestamp"]) for r in rows
              if "paged_attn_prefill" in r[key]), default=0)
    agg: dict = {}
    for r in rows:
        st = int(r["Start_Timestamp"])
        if st < t0:
            continue
        d = int(r["End_Timestamp"]) - st
        c, tot = agg.get(r[key], (0, 0))
        agg[r[key]] = (c + 1, tot + d)
    for name, (c, tot) in agg.items():
        yield (name, c, float(tot), None, None)


def main(path, out=None, title="kernel stats", top=30):
    if path.endswith("_kernel_trace.csv"):
        rows = list(_rows_trace_serving(path))
    else:
        rows = list(_rows_db(path) if path.endswith(".db") else _rows_csv(path))
    rows.sort(key=lambda r: -r[2])
    tot = sum(r[2] for r in rows)
    lines = [f"# {title}", "", f"source: `{path}`  total GPU kernel time {tot/1e6:.1f} ms", "",
             "| % | total ms | calls | avg us | VGPR | LDS B | kernel |",
             "|---:|---:|---:|---:|---:|---:|---|"]
    for name, calls, dur, vgpr, lds in rows[:top]:
        name = name.replace("|", "/")[:110]
        lines.append(f"| {100 * dur / tot:.2f} | {dur / 1e6:.2f} | {calls} | "
                     f"{dur / calls / 1e3:.2f} | {vgpr if vgpr is not None else ''} | "
                     f"{lds if lds is not None else ''} | `{name}` |")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None,
         sys.argv[3] if len(sys.argv) > 3 else "kernel stats")
