"""The conv kernels' small-int division (csrc/kernels/conv.hip qdiv, gemm.hip qdiv_s):
a / d == trunc((a + 0.5) * rcp(d)) in fp32 for 0 <= a < 2^20, d >= 1, with v_rcp_f32's result
anywhere within 1 ulp of 1/d.  Emulated here in numpy float32 over the ranges the kernels use
(thread / row / column indices < 2^16, divisors up to 2048) and a sample up to 2^20."""
import numpy as np


def _check(a: np.ndarray, d: int) -> None:
    r = np.float32(1.0) / np.float32(d)
    for rr in (np.nextafter(r, np.float32(0)), r, np.nextafter(r, np.float32(2))):
        q = ((a.astype(np.float32) + np.float32(0.5)) * np.float32(rr)).astype(np.int64)
        assert np.array_equal(q, a // d), (d, rr)


def test_qdiv_exact_small_operands():
    a = np.arange(0, 1 << 16, dtype=np.int64)
    for d in list(range(1, 300)) + [320, 500, 512, 576, 1024, 2047, 2048]:
        _check(a, d)


def test_qdiv_exact_to_2_pow_20_sampled():
    rng = np.random.default_rng(0)
    a = np.concatenate([rng.integers(0, 1 << 20, 200000), np.arange((1 << 20) - 4096, 1 << 20)]).astype(np.int64)
    for d in (1, 3, 7, 12, 25, 28, 144, 251, 1000, 4093):
        _check(a, d)
