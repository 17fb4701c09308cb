#!/usr/bin/env python3
"""Per-stage HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py.

    python tools/pmc_summary.py gpurun_out/prof_<tag> <steps_total> > profiles/pmc_traffic.json

steps_total: every proof the profiled bench ran -- warmup + steps + its untimed stage steps
(--stage-steps, default 2): `bench.py --no-extras --steps 2 --warmup 1` runs 5.

FETCH_SIZE / WRITE_SIZE are in KiB.  Correction per MI355X_MICROARCH.md (HBM section):
FETCH_SIZE on gfx950 reports half the bytes of wide coalesced reads -> x2; WRITE_SIZE as is.
Per stage (the TNS_PROF names bench.py reports), bytes per stage launch = the stage's kernels'
bytes in one step / the stage's launches in one step.
"""
import collections
import csv
import json
import sys

STAGES = {
    "msm_digits": (["k_scalar_bits", "k_u64_tables"], 2),  # the commitments (openings arrive canonical)
    "msm_sort": (["k_bs_", "k_scan_"], 4),
    "msm_accumulate": (["k_accumulate"], 4),
    "msm_fixup": (["k_fix_level", "k_bucket_fixup"], 4),
    "msm_reduce": (["k_reduce_level", "k_masked_sums", "k_sum_chunks", "k_set_sum"], 4),
    "open_scan": (["k_node_chain", "k_prod_reduce", "k_chain_", "k_node_finish", "k_sum_reduce", "k_node_quotient",
                   "k_quotient2"], 2),
    "sumcheck_round": (["k_sc_round", "k_sc_fold3", "k_sc_fold_tail", "k_sum_partials4"], None),
}


def per_kernel_last_step(path, counter, steps_total):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    by = collections.defaultdict(list)
    for r in rows:
        by[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    out = {}
    for k, v in by.items():
        per = len(v) // steps_total
        out[k] = (sum(v[len(v) - per:]) if per else 0.0, per)
    return out


def main():
    d, steps_total = sys.argv[1], int(sys.argv[2])
    import glob

    def find(sub):  # rocprofv3 may nest its output under host / pid directories
        hits = sorted(glob.glob(f"{d}/{sub}/**/run_counter_collection.csv", recursive=True))
        if not hits:
            raise SystemExit(f"no run_counter_collection.csv under {d}/{sub}")
        return hits[0]

    f = per_kernel_last_step(find("fetch"), "FETCH_SIZE", steps_total)
    w = per_kernel_last_step(find("write"), "WRITE_SIZE", steps_total)
    res = {"_note": "KiB counters x1024; FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md HBM); "
                    "per stage launch, one bench step (last of the run)"}
    for st, (pats, launches) in STAGES.items():
        fk = sum(v for k, (v, _) in f.items() if any(p in k for p in pats))
        wk = sum(v for k, (v, _) in w.items() if any(p in k for p in pats))
        if launches is None:  # sum-check: its fold launches
            launches = max(1, sum(n for k, (_, n) in f.items() if any(p in k for p in pats)))
        fb, wb = fk * 1024 * 2 / launches, wk * 1024 / launches
        res[st] = {"hbm_bytes_per_launch": fb + wb, "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                   "fetch_kib_raw_per_step": fk, "write_kib_raw_per_step": wk, "launches_per_step": launches}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
