"""Per-kernel MFMA busy fraction and wait / issue shares from two rocprofv3
--pmc passes (tools/gemm_pmc.sh, tools/pp_pmc.sh counter groups):

  MFMA_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
  WAIT_ANY, WAIT_INST_ANY, ACTIVE_INST_ANY as fractions of SQ_WAVE_CYCLES

    python tools/pmc_mfma.py <pass1 dir> <pass2 dir>
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    dur, cnt = {}, defaultdict(lambda: defaultdict(list))
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            dur[r.get("Dispatch_Id") or r.get("Dispatch_ID")] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            did = r.get("Dispatch_Id") or r.get("Dispatch_ID")
            cnt[r["Kernel_Name"]][r["Counter_Name"]].append((float(r["Counter_Value"]), dur.get(did, 0.0)))
    return cnt


def main():
    merged = defaultdict(dict)
    for d in sys.argv[1:]:
        for k, cs in load(d).items():
            for c, vals in cs.items():
                merged[k][c] = (sum(v for v, _ in vals) / len(vals), sum(t for _, t in vals) / len(vals))
    for k, cs in sorted(merged.items(), key=lambda kv: -max(t for _, t in kv[1].values())):
        us = max(t for _, t in cs.values())
        g = lambda n: cs.get(n, (float("nan"), 0))[0]  # noqa: E731
        wave = g("SQ_WAVE_CYCLES")
        busy = g("SQ_VALU_MFMA_BUSY_CYCLES") / (g("GRBM_GUI_ACTIVE") / 8 * 1024)
        print(k[:110])
        print(f"  us/call={us:.1f} MFMA_busy={busy:.3f} WAIT_ANY={g('SQ_WAIT_ANY') / wave:.3f} "
              f"WAIT_INST_ANY={g('SQ_WAIT_INST_ANY') / wave:.3f} ACTIVE_INST_ANY={g('SQ_ACTIVE_INST_ANY') / wave:.3f} "
              f"LDS_bank_conflict/LDS_active={g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_LDS_IDX_ACTIVE'), 1):.3f}")


if __name__ == "__main__":
    main()
