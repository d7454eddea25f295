"""Per-kernel summary of rocprofv3 --pmc passes (tools/pmc_profile.sh output).

    python tools/pmc_summary.py gpurun_out/pmc > profiles/<name>.md

Counters of every pass are summed per kernel over all dispatches, then a few derived
ratios are printed: LDS bank-conflict cycles per LDS-active cycle, VALU / LDS / VMEM
instructions per wave, MFMA busy share, HBM-side bytes per dispatch (FETCH_SIZE doubled:
on gfx950 it reports half the bytes of a wide coalesced read) and the L2 hit rate.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(root):
    sums = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    ns = defaultdict(dict)
    meta = {}
    for path in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        with open(path) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"]
                if k.startswith("__amd"):
                    continue
                sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((path, r["Dispatch_Id"]))
                ns[k][(path, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                meta[k] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"],
                           r["Scratch_Size"], r["Workgroup_Size"])
    return sums, disp, ns, meta


def short(name):
    name = name.replace("lgbm_amd::dev::", "").replace("(KArgs)", "")
    return name.replace("void ", "")[:60]


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    sums, disp, ns, meta = load(root)
    passes = max(1, len(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))))
    order = sorted(sums, key=lambda k: -sum(ns[k].values()))
    print("| kernel | disp/pass | VGPR | AGPR | LDS B | scratch | waves | VALU/wave | LDS/wave | VMEM rd/wave |"
          " LDS conflict / LDS active | wait share | MFMA insts | HBM rd+wr KB/disp | L2 hit |")
    print("|" + "---|" * 15)
    for k in order:
        c = sums[k]
        nd = max(1, len(disp[k]) // passes)
        waves = c.get("SQ_WAVES", 0.0) or 1.0
        conflict = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, c.get("SQ_LDS_IDX_ACTIVE", 0.0))
        wait = c.get("SQ_WAIT_ANY", 0.0) / max(1.0, c.get("SQ_WAVE_CYCLES", 0.0))
        hbm = (2 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) / nd
        hit = c.get("TCC_HIT_sum", 0.0) / max(1.0, c.get("TCC_HIT_sum", 0.0) + c.get("TCC_MISS_sum", 0.0))
        v, acc, _, lds, scr, _ = meta[k]
        print("| %s | %d | %s | %s | %s | %s | %.0f | %.1f | %.1f | %.1f | %.3f | %.2f | %.0f | %.1f | %.2f |" % (
            short(k), nd, v, acc, lds, scr, waves / nd, c.get("SQ_INSTS_VALU", 0) / waves,
            c.get("SQ_INSTS_LDS", 0) / waves, c.get("SQ_INSTS_VMEM_RD", 0) / waves, conflict, wait,
            c.get("SQ_INSTS_MFMA", 0), hbm, hit))


if __name__ == "__main__":
    main()
