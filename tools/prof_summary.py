#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV into markdown (for profiles/)."""
import csv
import sys


def main(path, out=None, title="kernel stats", top=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# {title}", "", f"source: `{path}`  total GPU kernel time {tot/1e6:.1f} ms", "",
             "| % | total ms | calls | avg us | kernel |", "|---:|---:|---:|---:|---|"]
    for r in rows[:top]:
        name = r["Name"].replace("|", "/")[:120]
        lines.append(f"| {float(r['Percentage']):.2f} | {float(r['TotalDurationNs'])/1e6:.2f} | "
                     f"{r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | `{name}` |")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None,
         sys.argv[3] if len(sys.argv) > 3 else "kernel stats")
