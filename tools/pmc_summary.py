#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter-collection CSVs into per-kernel markdown with derived
hardware metrics (for profiles/r2_pmc_*.md).

Input: one or more *_counter_collection.csv files (one row per dispatch x counter), e.g. from
  rocprofv3 --pmc SQ_WAVES GRBM_GUI_ACTIVE ... --output-format csv -d DIR -o run -- <cmd>
Counters of several passes (separate runs of the same workload) merge per kernel name.

Derived (when the counters are present; gfx950 conventions, MI355X_MICROARCH.md):
  * HBM read bytes = 2 x FETCH_SIZE KiB (FETCH_SIZE tallies 128-B streaming requests at 64 B
    on gfx950); read GB/s over the kernels' summed wall time
  * MFMA busy % = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 4 SIMD x 256 CU)
  * bf16 MFMA TFLOP/s = SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 / time
  * LDS bank-conflict % = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  * L2 hit % = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  * wave-time split = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
  * effective clock = GRBM_GUI_ACTIVE / 8 XCDs / wall time (per-XCD sum)

python tools/pmc_summary.py OUT.md TITLE file1.csv [file2.csv ...] [--calib REGEX=BYTES]
                            [--match REGEX ...]

--calib: a kernel whose HBM read bytes per call are known exactly (e.g. the decode attention
streams every cached K/V byte once); the ratio known / FETCH_SIZE of that kernel rescales
every row's read bytes, and is printed.  Without it the 2x rule above is used.
"""
import collections
import csv
import re
import sys

CUS, SIMDS_PER_CU, XCDS = 256, 4, 8


def load(paths):
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))
    wall = collections.defaultdict(dict)  # kernel -> {(file, dispatch): ns}
    for path in paths:
        for r in csv.DictReader(open(path)):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or "?"
            cname = r.get("Counter_Name") or r.get("Counter-Name")
            val = float(r.get("Counter_Value") or r.get("Counter-Value") or 0)
            disp = r.get("Dispatch_Id") or r.get("Dispatch-Id") or r.get("Correlation_Id")
            t0, t1 = r.get("Start_Timestamp"), r.get("End_Timestamp")
            if cname:
                ctr[name][cname] += val
            if t0 and t1:
                wall[name][(path, disp)] = int(t1) - int(t0)
            ctr[name]["__dispatch__" + path + str(disp)] = 1
    return ctr, wall


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "")[:90]


def derive(c: dict, wall_ns: float, calls: int, fetch_scale: float = 2.0) -> dict:
    out = {"calls": calls, "avg_us": wall_ns / max(calls, 1) / 1e3}
    sec = wall_ns / 1e9
    if "FETCH_SIZE" in c and sec > 0:
        rd = fetch_scale * c["FETCH_SIZE"] * 1024
        out["hbm_read_GB"] = rd / 1e9
        out["read_TBps"] = rd / sec / 1e12
    if "WRITE_SIZE" in c and sec > 0:
        out["write_TBps"] = c["WRITE_SIZE"] * 1024 / sec / 1e12
    g = c.get("GRBM_GUI_ACTIVE", 0)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and g:
        # GRBM_GUI_ACTIVE sums the 8 XCDs' counters: per-XCD cycles = g / 8
        out["mfma_busy_%"] = 100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / XCDS * SIMDS_PER_CU * CUS)
    if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in c and sec > 0:
        out["bf16_TFLOPs"] = c["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 / sec / 1e12
    if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_conflict_%"] = 100 * c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
    if "TCC_HIT_sum" in c and (c["TCC_HIT_sum"] + c.get("TCC_MISS_sum", 0)):
        out["l2_hit_%"] = 100 * c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c.get("TCC_MISS_sum", 0))
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        for k, lab in (("SQ_WAIT_ANY", "wait_%"), ("SQ_WAIT_INST_ANY", "issue_stall_%"),
                       ("SQ_ACTIVE_INST_ANY", "active_%")):
            if k in c:
                out[lab] = 100 * c[k] / wc
    if g and sec > 0:
        out["clock_GHz"] = g / XCDS / sec / 1e9
    if "SQ_WAVES" in c:
        out["waves"] = c["SQ_WAVES"]
    return out


def main(argv):
    out_md, title, rest = argv[0], argv[1], argv[2:]
    pats = []
    calib = None
    if "--calib" in rest:
        i = rest.index("--calib")
        calib = rest[i + 1]
        rest = rest[:i] + rest[i + 2:]
    if "--match" in rest:
        i = rest.index("--match")
        pats = [re.compile(p) for p in rest[i + 1:]]
        rest = rest[:i]
    ctr, wall = load(rest)
    scale, note = 2.0, "FETCH_SIZE x 2 (gfx950 rule, MI355X_MICROARCH.md)"
    if calib:
        rx, nbytes = calib.rsplit("=", 1)
        for name, c in ctr.items():
            if re.search(rx, name) and c.get("FETCH_SIZE"):
                calls = sum(1 for k in c if k.startswith("__dispatch__"))
                scale = float(nbytes) * calls / (c["FETCH_SIZE"] * 1024)
                note = (f"calibrated on `{short(name)}`: {float(nbytes) / 1e6:.1f} MB known per "
                        f"call = FETCH_SIZE x {scale:.2f}")
                break
    rows = []
    for name, c in ctr.items():
        if pats and not any(p.search(name) for p in pats):
            continue
        calls = sum(1 for k in c if k.startswith("__dispatch__"))
        w = sum(wall[name].values())
        rows.append((w, name, derive(c, w, calls, scale)))
    rows.sort(key=lambda r: -r[0])
    cols = ["calls", "avg_us", "read_TBps", "write_TBps", "hbm_read_GB", "mfma_busy_%",
            "bf16_TFLOPs", "lds_conflict_%", "l2_hit_%", "wait_%", "issue_stall_%", "active_%",
            "clock_GHz"]
    lines = [f"# {title}", "", "sources: " + ", ".join(f"`{p}`" for p in rest), "",
             f"HBM read bytes: {note}", "",
             "| kernel | " + " | ".join(cols) + " |", "|---|" + "---:|" * len(cols)]
    for w, name, d in rows[:25]:
        cells = []
        for k in cols:
            v = d.get(k)
            cells.append("" if v is None else (f"{v:.0f}" if k == "calls" else f"{v:.2f}"))
        lines.append(f"| `{short(name)}` | " + " | ".join(cells) + " |")
    open(out_md, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1:])
