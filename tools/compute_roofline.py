"""Compute (VALU-issue) roofline of the AEAD kernels: the minimum time one launch
needs to ISSUE its vector instructions, from the per-packet instruction mix and
the measured per-instruction issue costs on MI355X.

Issue costs (SIMD-cycles per wave64 instruction, 4 waves per SIMD):
  * "simple" ops -- v_add_u32, v_xor_b32, v_or/and_b32, v_lshrrev_b32, v_mov,
    v_bitop3 -- 2 cycles when two waves of a SIMD issue them in step; every
    other op (v_alignbit_b32, v_mad_u64_u32, v_add_co/addc_co, v_lshrrev_b64,
    v_lshlrev_b32, ...) 4 cycles (profiles/r01_microbench_valu.txt,
    r01_microbench_valu3.txt, r01_microbench_valu4.txt);
  * one ChaCha20 block, phase-locked 8 add + 8 xor + 8 alignbit steps with a
    barrier per step (wg_crypto.h chacha20_block2_sync): 2376.6 SIMD-cycles per
    wave-block measured (profiles/r01_microbench_chacha2.txt, "asm,
    barrier/step"); the pure issue model is 80 quarter-rounds x 4 ARX steps x
    (2 + 2 + 4) = 2560, the first column round partly runs on the SALU.

Instruction mix per packet and direction (wg_aead.hip / wg_crypto.h):
  * ChaCha20 blocks: 2 per 128-byte round that holds text (2r+1, 2r+2, computed
    as a pair even when the text ends in the first) + 1 Poly1305 key block;
  * Poly1305 blocks: ceil(P/16) text blocks + 1 length block, each 21
    v_mad_u64_u32 + 10 carry adds + 4 v_lshrrev_b64 (4-cycle ops) + 4 simple
    ops (the 2^130 fold) = 148 SIMD-cycles (poly_block);
  * keystream XOR: 4 v_xor_b32 per 16-byte chunk = 8 SIMD-cycles.
Everything else (staging address math, tag, header checks) is left out: this
is a floor.  The model's VALU instruction count is returned too, so it can be
checked against the PMC SQ_INSTS_VALU / SQ_WAVES of the same launch.
"""
from __future__ import annotations

import math

CHACHA_WAVE_BLOCK_CYCLES = 2376.6  # profiles/r01_microbench_chacha2.txt
POLY_BLOCK_CYCLES = 35 * 4 + 4 * 2   # wg_crypto.h poly_block
XOR_CHUNK_CYCLES = 4 * 2
SIMDS = 1024                          # 256 CUs x 4 SIMDs
PEAK_CLOCK_GHZ = 2.4

CHACHA_BLOCK_INSTR = 80 * 4 * 3 + 16  # ARX ops + feed-forward adds
POLY_BLOCK_INSTR = 39
XOR_CHUNK_INSTR = 4


def packet_mix(P: int) -> dict:
    """Work one lane does for one packet of payload P in one direction."""
    text_rounds = math.ceil(P / 128) if P > 0 else 0
    chacha = 2 * text_rounds + 1
    poly = math.ceil(P / 16) + 1
    chunks = math.ceil(P / 16)
    cycles = chacha * CHACHA_WAVE_BLOCK_CYCLES + poly * POLY_BLOCK_CYCLES + chunks * XOR_CHUNK_CYCLES
    instr = chacha * CHACHA_BLOCK_INSTR + poly * POLY_BLOCK_INSTR + chunks * XOR_CHUNK_INSTR
    return {"chacha_blocks": chacha, "poly_blocks": poly, "wave_cycles": cycles, "valu_instr": instr}


def launch_floor(sizes, clock_ghz: float | None = None) -> dict:
    """VALU-issue floor of one seal or open launch over packets of the given
    payload sizes (an int with a count, or an iterable of sizes).  One wave
    carries 64 packets, so a launch costs sum(wave_cycles) / 64 SIMD-cycles of
    issue, spread over all SIMDs."""
    if isinstance(sizes, tuple):  # (P, n)
        P, n = sizes
        m = packet_mix(P)
        cyc = m["wave_cycles"] * n / 64
        instr = m["valu_instr"] * n / 64
    else:
        cyc = instr = 0.0
        for P, cnt in sizes.items():
            m = packet_mix(int(P))
            cyc += m["wave_cycles"] * cnt / 64
            instr += m["valu_instr"] * cnt / 64
    per_simd = cyc / SIMDS
    out = {"simd_cycles_per_simd": round(per_simd),
           "floor_ms_at_2p4GHz": round(per_simd / (PEAK_CLOCK_GHZ * 1e9) * 1e3, 4),
           "model_valu_instr_per_64_packets": round(instr * 64 / max(1, sum_count(sizes)), 1)}
    if clock_ghz:
        out["floor_ms_at_profiled_clock"] = round(per_simd / (clock_ghz * 1e9) * 1e3, 4)
    return out


def sum_count(sizes) -> int:
    if isinstance(sizes, tuple):
        return sizes[1]
    return int(sum(sizes.values()))


if __name__ == "__main__":
    import json
    print(json.dumps({"config2_per_launch": launch_floor((1350, 1 << 20), 1.78),
                      "packet_1350": packet_mix(1350)}, indent=1))
