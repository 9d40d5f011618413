"""Compute (VALU-issue) roofline of the AEAD kernels: the minimum time one launch
needs to ISSUE its vector instructions, from the per-packet instruction mix and
the measured issue cost of the phase-locked ChaCha20 steps on MI355X.

Issue cost.  One ChaCha20 block in the phase-locked form (8 add + 8 xor + 8
alignbit per step, s_barrier per step, 4 waves per SIMD) measured 2376.6
SIMD-cycles per wave-block (profiles/r01_microbench_chacha2.txt, "asm,
barrier/step wg1024"; the product's 512-thread shape measured 2612.3 -- the
floor keeps the faster figure).  That microbenchmark block issues 984 VALU
instructions (all 20 rounds in asm, 8 feed-forward adds, 16 xors), so the
model prices a ChaCha20 VALU instruction at 2376.6 / 984 SIMD-cycles.
Poly1305 (21 v_mad_u64_u32 + 10 carry adds + 4 v_lshrrev_b64, all 4-cycle
ops, + 4 simple ops) = 148 SIMD-cycles per block; the keystream XOR 4 simple
ops = 8 SIMD-cycles per 16-byte chunk.

Instruction mix per packet and direction (wg_crypto.h chacha20_block2_sync /
chacha20_block_sync, wg_aead.hip run_wave).  A block is 80 quarter-rounds x 12
ARX ops = 960 + feed-forward adds (word 13 starts at 0: 15 adds).  What the
kernels take off the VALU, counted here:
  * uniform batches (one session key in SGPRs, configs 2 / 5): in the first
    column round, columns 0 and 1 of block 2r+1 and column 0 of block 2r+2 are
    wave-uniform (sigma, key, block number, word 13 = 0) and run on the SALU,
    as do the first adds of columns 2 and 3 (26 ops); columns 1-3 of block
    2r+2 equal those of block 2r+1 and are not recomputed (36 ops); the first
    diagonal round runs its all-common ops once (4 ops).  Per block pair:
    2 x 975 - 26 - 36 - 4 = 1884 -> 942 per keystream block; the Poly1305 key
    block (single, uniform): 975 - 26 = 949;
  * per-lane keys (descriptor kernels, configs 3 / 4): every op is per-lane
    (the key is in VGPRs), no shared words: 975 per block.
Poly1305: ceil(P/16) text blocks + 1 length block, 39 VALU each.  XOR: 4 per
16-byte chunk.  Everything else (staging address math, tag, header checks)
is left out: this is a floor, and its instruction count must stay at or below
the PMC SQ_INSTS_VALU / SQ_WAVES of the same launch (bench.py reports both).
"""
from __future__ import annotations

import math

CHACHA_MICROBENCH_WAVE_BLOCK_CYCLES = 2376.6  # profiles/r01_microbench_chacha2.txt
CHACHA_MICROBENCH_BLOCK_INSTR = 960 + 8 + 16  # ARX + feed-forward adds + xor accumulate
CHACHA_CYCLES_PER_INSTR = CHACHA_MICROBENCH_WAVE_BLOCK_CYCLES / CHACHA_MICROBENCH_BLOCK_INSTR
POLY_BLOCK_CYCLES = 35 * 4 + 4 * 2   # wg_crypto.h poly_block
XOR_CHUNK_CYCLES = 4 * 2
SIMDS = 1024                          # 256 CUs x 4 SIMDs
PEAK_CLOCK_GHZ = 2.4

BLOCK_FULL_INSTR = 80 * 12 + 15       # per-lane block: ARX + feed-forward
PAIR_UNIFORM_INSTR = 2 * BLOCK_FULL_INSTR - 26 - 36 - 4
KEYBLOCK_UNIFORM_INSTR = BLOCK_FULL_INSTR - 26
POLY_BLOCK_INSTR = 39
XOR_CHUNK_INSTR = 4


def packet_mix(P: int, per_lane_keys: bool = False) -> dict:
    """Work one lane does for one packet of payload P in one direction."""
    pairs = math.ceil(P / 128) if P > 0 else 0   # two keystream blocks per 128-byte round
    if per_lane_keys:
        chacha_instr = (2 * pairs + 1) * BLOCK_FULL_INSTR
    else:
        chacha_instr = pairs * PAIR_UNIFORM_INSTR + KEYBLOCK_UNIFORM_INSTR
    poly = math.ceil(P / 16) + 1
    chunks = math.ceil(P / 16)
    cycles = (chacha_instr * CHACHA_CYCLES_PER_INSTR + poly * POLY_BLOCK_CYCLES
              + chunks * XOR_CHUNK_CYCLES)
    instr = chacha_instr + poly * POLY_BLOCK_INSTR + chunks * XOR_CHUNK_INSTR
    return {"chacha_blocks": 2 * pairs + 1, "chacha_instr": chacha_instr, "poly_blocks": poly,
            "wave_cycles": cycles, "valu_instr": instr}


def launch_floor(sizes, clock_ghz: float | None = None, per_lane_keys: bool = False) -> dict:
    """VALU-issue floor of one seal or open launch over packets of the given
    payload sizes ({P: count} or a (P, n) tuple).  One wave carries 64
    packets, so a launch costs sum(wave_cycles) / 64 SIMD-cycles of issue,
    spread over all SIMDs."""
    items = [sizes] if isinstance(sizes, tuple) else list(sizes.items())
    cyc = instr = 0.0
    for P, cnt in items:
        m = packet_mix(int(P), per_lane_keys)
        cyc += m["wave_cycles"] * cnt / 64
        instr += m["valu_instr"] * cnt / 64
    n = sum(c for _, c in items)
    per_simd = cyc / SIMDS
    out = {"simd_cycles_per_simd": round(per_simd),
           "floor_ms_at_2p4GHz": round(per_simd / (PEAK_CLOCK_GHZ * 1e9) * 1e3, 4),
           "model_valu_instr_per_64_packets": round(instr * 64 / max(1, n), 1),
           "keys": "per-lane (VGPR)" if per_lane_keys else "uniform (SGPR)"}
    if clock_ghz:
        out["floor_ms_at_clock"] = round(per_simd / (clock_ghz * 1e9) * 1e3, 4)
    return out


if __name__ == "__main__":
    import json
    print(json.dumps({"config2_per_launch": launch_floor((1350, 1 << 20), 1.96),
                      "config4_per_launch": launch_floor((1350, 1 << 24), 1.92, per_lane_keys=True),
                      "packet_1350": packet_mix(1350)}, indent=1))
