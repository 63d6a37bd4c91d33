"""Host-side checks of arithmetic identities the env kernel relies on (no GPU).

small_div (marl-scheduling_amd/csrc/env_kernels.hip): x / d for 0 <= x < 256, 1 <= d < 256 as
floor((x + 1/2) * rcp(d)) in float32. The device reciprocal (v_rcp_f32) is not correctly rounded,
so the identity is checked with the reciprocal perturbed by up to +-2 ulp."""
import numpy as np


def test_small_div_exact_with_inexact_reciprocal():
    x = np.arange(256, dtype=np.float32) + np.float32(0.5)
    want = np.arange(256)
    for d in range(1, 256):
        r = np.float32(1) / np.float32(d)
        for k in range(-2, 3):
            rk = r
            step = np.float32(2) if k > 0 else np.float32(0)
            for _ in range(abs(k)):
                rk = np.nextafter(rk, step)
            q = np.floor(x * np.float32(rk)).astype(np.int64)  # float32 product, round to nearest
            assert np.array_equal(q, want // d), (d, k)
