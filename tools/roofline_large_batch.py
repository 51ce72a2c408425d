#!/usr/bin/env python3
"""Roofline of the large-batch training step (BASELINE config 5: global batch 8192, fp16; per-rank
batch 1024 on 8 GPUs) for the two designs the verdicts asked to compare:

* TILE  -- csrc/kernels/lenet_tile.hip: one workgroup per CU walks tiles of 4 samples through the
  whole network in LDS (64 KB of weight images + 4 samples' activations), the conv weight
  gradients accumulating in registers; activations never touch HBM.
* LAYER -- a batched layer-wise path: each layer (or fused group of layers) is its own kernel over
  the whole batch, its GEMM M = batch x pixels, activations handed between kernels through HBM.

For each kernel the bound is max(MFMA issue, LDS operand traffic, HBM traffic) at the chip's
rates; the step adds the update kernel (measured) and the kernel boundaries (measured price).

    python tools/roofline_large_batch.py [--batch 8192 1024] [--clock-ghz 2.3]

Hardware numbers: /opt/skills/guides/MI355X_MICROARCH.md (256 CUs x 4 SIMDs; v_mfma_f32_16x16x32_f16
16 cycles back to back on one SIMD; LDS 256 B/clk/CU for ds_read_b64/b128, ~150 TB/s chip-wide;
HBM 6.3 TB/s achievable; dependent kernel boundary 1.45-1.9 us).  Per-tile MFMA counts of TILE are
from the kernel's stage comments (lenet_tile.hip:14-22); measured times from profiles/tile_r4.md
and profiles/r4/stages_r4f8_stage_tile1024.txt.
"""
from __future__ import annotations

import argparse
import math

CUS, SIMDS = 256, 4
MFMA_CYC = 16               # v_mfma_f32_16x16x32_f16, cycles per instruction on one SIMD
FRAG = 16 * 32 * 2          # bytes of one 16x32 fp16 operand fragment (A or B)
LDS_BPC = 256               # LDS bytes per clock per CU (ds_read_b128)
HBM_BPS = 6.3e12            # achievable HBM bytes/s
BOUNDARY_US = 1.6           # dependent kernel boundary inside a graph
UPDATE_US = {1024: 4.7 + 2.5, 8192: 10.3}  # lenet_update FC-role span (+ CONV tail at 1024), tile_r4.md §1


def tiles(n: int, t: int) -> int:
    return math.ceil(n / t)


def layer_kernels() -> list[dict]:
    """Per-sample work of the layer-wise design, three kernels (fp16 activations).

    F  forward + loss + fc backward + dP2 (conv1, pool1, conv2, Dropout2d, pool2, fc1, fc2, loss,
       dlogits, dZ1, dP2 -> dL/dconv2): writes what the conv backward needs.
    B  conv2 wgrad + conv2 dgrad + pool1 backward + conv1 wgrad, dW in registers across samples.
    (U  lenet_update as today: reads the fc vectors + one slab row per workgroup.)

    MFMA counts use 16x16x32 tiles with channel padding (10 -> 16, 20 -> 32) as the tile kernel
    does; LDS bytes count the operand fragments that stream from LDS (weights that every sample
    reuses are held in registers: the dgrad's W2 image, conv1 / conv2 forward B operands)."""
    conv1_f = tiles(576, 16) * 1 * 1                    # M 576 px, N 10->16, K 25->32
    conv2_f = tiles(64, 16) * 2 * tiles(250, 32)        # M 64 px, N 20->32, K 250->256
    fc = 2 * 4 * 10 / 16 + 20 * 2 / 16                  # fc1 fwd, dP2: per 16 samples
    dgrad = tiles(144, 16) * 1 * tiles(500, 32)         # M 144 px, N 10->16, K 500->512
    wgrad2 = 2 * 26 * tiles(64, 32)                     # M 20->32 (2), N 26 taps x 16 ch, K 64 px
    wgrad1 = 1 * 2 * tiles(576, 32)                     # M 10->16, N 26->32, K 576 px
    # HBM bytes per sample (fp16 activations, u8 pool argmax, u8 pixels)
    f_in = 784 + 8                                      # pixels + label
    f_out = 1440 * 2 + 1440 + 1280 * 2 + 464 * 2        # P1, pool1 argmax, dL/dconv2, fc vectors
    b_in = 1440 * 2 + 1440 + 1280 * 2 + 784             # P1, argmax, dL/dconv2, pixels
    return [
        {"name": "F (fwd + fc bwd + dP2)", "mfma": conv1_f + conv2_f + fc,
         "lds": (conv1_f + conv2_f + fc) * FRAG, "hbm": f_in + f_out},
        {"name": "B (conv2 wgrad+dgrad, conv1 wgrad)", "mfma": dgrad + wgrad2 + wgrad1,
         # dgrad: A streams (B = W2 in registers); wgrad2: per 32-px K-block 2 A + 26 B reads for
         # 52 MFMAs; wgrad1: A and B per MFMA
         "lds": dgrad * FRAG + tiles(64, 32) * (2 + 26) * FRAG + wgrad1 * 2 * FRAG, "hbm": b_in},
    ]


def bound_us(per_sample: dict, batch: int, ghz: float) -> dict:
    spc = batch / CUS                                   # samples per CU
    mfma = per_sample["mfma"] * spc * MFMA_CYC / SIMDS / (ghz * 1e3)
    lds = per_sample["lds"] * spc / LDS_BPC / (ghz * 1e3)
    hbm = per_sample["hbm"] * batch / HBM_BPS * 1e6
    return {"mfma_us": mfma, "lds_us": lds, "hbm_us": hbm, "bound_us": max(mfma, lds, hbm)}


def tile_design(batch: int, ghz: float) -> dict:
    """TILE at its own bounds: ~1,900 MFMAs and ~1.6 MB of LDS operand reads per 4-sample tile
    (stage 6 alone ~1.1k MFMAs / ~1 MB, tile_r4.md §4), no activation HBM traffic."""
    spc = batch / CUS
    t = math.ceil(spc / 4)
    mfma = t * 1900 * MFMA_CYC / SIMDS / (ghz * 1e3)
    lds = t * 1.6e6 / LDS_BPC / (ghz * 1e3)
    hbm = batch * (784 + 464 * 2) / HBM_BPS * 1e6
    return {"mfma_us": mfma, "lds_us": lds, "hbm_us": hbm, "bound_us": max(mfma, lds, hbm)}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[8192, 1024])
    ap.add_argument("--clock-ghz", type=float, default=2.3)
    a = ap.parse_args(argv)
    measured = {8192: {"tile": 117.3, "step": 136.0}, 1024: {"tile": 20.0, "step": 29.3}}
    print("| batch | design | kernel | MFMA µs | LDS µs | HBM µs | bound µs |")
    print("|---:|---|---|---:|---:|---:|---:|")
    for b in a.batch:
        tb = tile_design(b, a.clock_ghz)
        print(f"| {b} | TILE | lenet_tile | {tb['mfma_us']:.1f} | {tb['lds_us']:.1f} | {tb['hbm_us']:.1f} | "
              f"{tb['bound_us']:.1f} |")
        tot = 0.0
        for k in layer_kernels():
            r = bound_us(k, b, a.clock_ghz)
            tot += r["bound_us"]
            print(f"| {b} | LAYER | {k['name']} | {r['mfma_us']:.1f} | {r['lds_us']:.1f} | {r['hbm_us']:.1f} | "
                  f"{r['bound_us']:.1f} |")
        upd = UPDATE_US.get(b, UPDATE_US[8192])
        tile_step = tb["bound_us"] + upd + 2 * BOUNDARY_US
        layer_step = tot + upd + 3 * BOUNDARY_US
        m = measured.get(b, {})
        print(f"| {b} | step bound | TILE {tile_step:.1f} µs, LAYER {layer_step:.1f} µs (update {upd} µs + "
              f"boundaries); measured TILE kernel {m.get('tile', '-')} µs, step {m.get('step', '-')} µs | | | | |")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
