"""Per-kernel byte / MFMA table from a tools/pmc_by_dispatch.py listing
(FETCH_SIZE, WRITE_SIZE, SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE columns):
us per step, achieved HBM TB/s (FETCH_SIZE doubled: gfx950 counts a wide
coalesced read at half its bytes), MFMA busy, read / write MiB per call.

    python tools/pmc_bytes_table.py gpurun_out/r5_rn_pmc.txt --steps 5 [--top 30]
"""
import argparse
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = []
    for line in open(a.path):
        m = re.match(r"\s*(\d+) x\s+([\d.]+) us grid=\s*(\d+)", line)
        tot = re.search(r"total\(x2 fetch\)=([\d.]+)TB/s\s+(.*)$", line)
        if not m or not tot:
            continue
        n, us = int(m[1]), float(m[2])
        mb = float(re.search(r"SQ_VALU_MFMA_BUSY_CYCLES=([\d.e+]+)", line)[1])
        ga = float(re.search(r"GRBM_GUI_ACTIVE=([\d.e+]+)", line)[1])
        rd = 2 * float(re.search(r"FETCH_SIZE=([\d.]+)MiB", line)[1])
        wr = float(re.search(r"WRITE_SIZE=([\d.]+)MiB", line)[1])
        busy = mb / (ga / 8 * 1024) if ga > 0 else 0.0  # per-SIMD MFMA-busy share (256 CUs x 4 SIMDs)
        name = re.sub(r"\(.*", "", tot[2].strip())
        for s in ("void ", "dcp::kern::", "(anonymous namespace)::", "at::native::"):
            name = name.replace(s, "")
        rows.append((n * us / a.steps, n // a.steps, us, float(tot[1]), busy, rd, wr, name))
    rows.sort(reverse=True)
    print(f"{'us/step':>8} {'calls':>5} {'us/call':>8} {'TB/s':>5} {'MFMA':>5} {'rd MiB':>7} {'wr MiB':>7}  kernel")
    for r in rows[: a.top]:
        print(f"{r[0]:8.0f} {r[1]:5d} {r[2]:8.1f} {r[3]:5.2f} {r[4]:5.2f} {r[5]:7.0f} {r[6]:7.0f}  {r[7][:80]}")
    tot = sum(r[0] for r in rows)
    bound = sum(r[0] for r in rows if r[3] >= 4.5)
    print(f"# {tot:.0f} us/step in the listed kernels; {bound:.0f} us ({bound / tot:.0%}) in kernels at >= 4.5 TB/s "
          f"(HBM-bound: ~6.3 TB/s achievable)")


if __name__ == "__main__":
    main()
