"""Summarise rocprofv3 rocpd databases into the committed profiles/ files.

  python tools/prof_summary.py <tag>
reads gpurun_out/prof_<tag>/run_results.db (--kernel-trace --stats) and the
two PMC passes gpurun_out/pmc_{fetch,write}_<tag>/run_results.db, writes
profiles/<tag>_kernel_stats.csv, profiles/<tag>_pmc.csv and
profiles/<tag>_summary.json (per-launch HBM traffic of each kernel, with the
gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE counts
half the bytes of 16-B-per-lane reads, so it is doubled; WRITE_SIZE as is).
"""
import csv
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split("(")[0]


def kernel_stats(db):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    # rocpd top_kernels durations are in microseconds
    return [dict(kernel=short(r[0]), calls=r[1], total_ms=r[2] / 1e3, avg_ms=r[3] / 1e3, pct=r[4]) for r in rows]


def pmc(db, counter):
    c = sqlite3.connect(db)
    out = {}
    for name, val, n in c.execute("select kernel_name, sum(value), count(*) from counters_collection "
                                  "where counter_name = ? group by kernel_name", (counter,)):
        k = short(name)
        s = out.setdefault(k, [0.0, 0])
        s[0] += val
        s[1] += n
    print(f"  {counter}: {len(out)} kernels", flush=True)
    return out


def db(kind, tag):
    """rocpd database of one pass: $PROF_DB_ROOT/<kind>/ (tools/prof_passes.sh) or
    gpurun_out/<kind>_<tag>/ (older layout)"""
    root = os.environ.get("PROF_DB_ROOT")
    if root:
        return os.path.join(root, kind, "run_results.db")
    return os.path.join(ROOT, "gpurun_out", f"{kind}_{tag}", "run_results.db")


def main(tag, outdir=None):
    ks = kernel_stats(db("prof", tag))
    prof = outdir or os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    with open(os.path.join(prof, f"{tag}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["kernel", "calls", "total_ms", "avg_ms", "pct"])
        w.writeheader()
        for r in ks:
            w.writerow(r)
    fetch = pmc(db("pmc_fetch", tag), "FETCH_SIZE")
    write = pmc(db("pmc_write", tag), "WRITE_SIZE")
    per = {}
    with open(os.path.join(prof, f"{tag}_pmc.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches", "FETCH_SIZE_KB_per_dispatch", "WRITE_SIZE_KB_per_dispatch",
                    "hbm_bytes_per_dispatch_corrected"])
        for k in sorted(set(fetch) | set(write)):
            fk = fetch.get(k, [0.0, 1])
            wk = write.get(k, [0.0, 1])
            f_kb, w_kb = fk[0] / fk[1], wk[0] / wk[1]
            corrected = 2.0 * f_kb * 1024 + w_kb * 1024
            per[k] = dict(dispatches=fk[1], fetch_kb=f_kb, write_kb=w_kb, hbm_bytes=corrected)
            w.writerow([k, fk[1], f"{f_kb:.3f}", f"{w_kb:.3f}", f"{corrected:.0f}"])
    extra = {}
    mdb = db("pmc_mfma", tag)
    if os.path.exists(mdb):
        try:
            for cn in ("SQ_INSTS_VALU_MFMA_F64", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES",
                       "SQ_INSTS_VALU_FMA_F64", "GRBM_GUI_ACTIVE"):
                for k, (v, n) in pmc(mdb, cn).items():
                    extra.setdefault(k, {})[cn + "_per_dispatch"] = v / n
        except sqlite3.Error as e:  # a pass killed at its time limit leaves a partial database
            print(f"  MFMA pass database unreadable ({e}); pmc_issue left empty", flush=True)
            extra = {}
    summary = dict(tag=tag, kernels=ks, pmc_per_dispatch=per, pmc_issue=extra,
                   note="rocprofv3 --kernel-trace --stats and separate --pmc passes (FETCH_SIZE, WRITE_SIZE, "
                        "MFMA/issue counters) of the same `python3 bench.py` command; FETCH_SIZE doubled per the "
                        "gfx950 calibration")
    with open(os.path.join(prof, f"{tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: v for k, v in per.items() if k.startswith("k_")}, indent=1))
    for r in ks[:4]:
        print(r)


def one_pass(kind, tag, out):
    """one pass of a long command per GPU call (each under the call's time limit):
    its partial summary (kernel stats, or one counter's per-kernel sums) as JSON"""
    d = db(kind, tag)
    if kind == "prof":
        res = {"kernels": kernel_stats(d)}
    else:
        counter = {"pmc_fetch": "FETCH_SIZE", "pmc_write": "WRITE_SIZE"}[kind]
        res = {"counter": counter, "sums": pmc(d, counter)}
    with open(out, "w") as f:
        json.dump(res, f)


def merge(tag, parts, outdir=None):
    """profiles/<tag>_{kernel_stats.csv,pmc.csv,summary.json} from one_pass outputs"""
    prof = outdir or os.path.join(ROOT, "profiles")
    ks, fetch, write = [], {}, {}
    for pth in parts:
        with open(pth) as f:
            r = json.load(f)
        if "kernels" in r:
            ks = r["kernels"]
        elif r["counter"] == "FETCH_SIZE":
            fetch = r["sums"]
        else:
            write = r["sums"]
    with open(os.path.join(prof, f"{tag}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["kernel", "calls", "total_ms", "avg_ms", "pct"])
        w.writeheader()
        for r in ks:
            w.writerow(r)
    per = {}
    with open(os.path.join(prof, f"{tag}_pmc.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches", "FETCH_SIZE_KB_per_dispatch", "WRITE_SIZE_KB_per_dispatch",
                    "hbm_bytes_per_dispatch_corrected"])
        for k in sorted(set(fetch) | set(write)):
            fk = fetch.get(k, [0.0, 1])
            wk = write.get(k, [0.0, 1])
            f_kb, w_kb = fk[0] / fk[1], wk[0] / wk[1]
            corrected = 2.0 * f_kb * 1024 + w_kb * 1024
            per[k] = dict(dispatches=fk[1], fetch_kb=f_kb, write_kb=w_kb, hbm_bytes=corrected)
            w.writerow([k, fk[1], f"{f_kb:.3f}", f"{w_kb:.3f}", f"{corrected:.0f}"])
    summary = dict(tag=tag, kernels=ks, pmc_per_dispatch=per, pmc_issue={},
                   note="rocprofv3 --kernel-trace --stats and separate --pmc passes (FETCH_SIZE, WRITE_SIZE) of "
                        "the same `python3 bench.py` command, each pass in a GPU call of its own (one pass "
                        "nearly fills a call's time limit); FETCH_SIZE doubled per the gfx950 calibration")
    with open(os.path.join(prof, f"{tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: v for k, v in per.items() if "gemm" in k}, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--pass":
        one_pass(sys.argv[2], sys.argv[3], sys.argv[4])
    elif len(sys.argv) > 1 and sys.argv[1] == "--merge":
        merge(sys.argv[2], sys.argv[3:])
    else:
        main(sys.argv[1] if len(sys.argv) > 1 else "r01", sys.argv[2] if len(sys.argv) > 2 else None)
