"""Derived per-kernel metrics from tools/pmc.sh output (pmc_summary.py text): MFMA busy share of the
SIMD cycles, VALU / LDS instruction shares, LDS bank-conflict cycles per LDS instruction, waits, L2
hit rate and the memory-side request bytes (TCC_EA0_RDREQ / WRREQ x 64 B; on gfx950 a wide
streaming read is counted at half its bytes, MI355X_MICROARCH.md).

    python tools/pmc_derived.py gpurun_out/<tag>/pmc.txt [name-filter ...]"""
import sys


def parse(path):
    out, cur = {}, None
    for line in open(path):
        if not line.startswith("    "):
            cur = line.strip()
            out[cur] = {}
        elif cur is not None:
            k, v = line.split()
            out[cur][k] = float(v)
    return out


def main():
    d = parse(sys.argv[1])
    filt = sys.argv[2:]
    print(f"{'kernel':58s} {'MFMA%':>6s} {'VALU/MFMA':>9s} {'LDSconf/LDSinst':>15s} {'wait%':>6s} {'L2hit%':>6s} "
          f"{'RD MB':>8s} {'WR MB':>8s}")
    for k, c in d.items():
        if filt and not any(f in k for f in filt):
            continue
        if "MFMA" not in k.upper() and c.get("SQ_INSTS_MFMA", 0) == 0:
            continue
        xcd_cycles = c.get("GRBM_GUI_ACTIVE", 0) / 8.0
        simd_cycles = xcd_cycles * 256 * 4
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / simd_cycles * 100 if simd_cycles else 0
        vpm = c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_INSTS_MFMA", 1), 1)
        conf = c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_INSTS_LDS", 1), 1)
        wait = c.get("SQ_WAIT_ANY", 0) / max(c.get("SQ_WAVE_CYCLES", 1), 1) * 100
        hit = c.get("TCC_HIT_sum", 0) / max(c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0), 1) * 100
        rd = c.get("TCC_EA0_RDREQ_sum", 0) * 64 / 1e6
        wr = c.get("TCC_EA0_WRREQ_sum", 0) * 64 / 1e6
        print(f"{k[:58]:58s} {mfma:6.1f} {vpm:9.2f} {conf:15.2f} {wait:6.1f} {hit:6.1f} {rd:8.1f} {wr:8.1f}")


if __name__ == "__main__":
    main()
