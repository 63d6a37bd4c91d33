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


def test_mulhi_quotient_with_one_correction():
    """k_act_pair's row -> (replica, unit) and unit -> agent quotients (policy_kernels.hip
    core_row_of): q = umulhi(x, floor((2^32 - 1) / d)), plus one if (q + 1) * d <= x, equals x // d
    for every x < 2^31 (checked on a dense low range and random draws, for the divisors in use)."""
    rng = np.random.default_rng(7)
    xs = np.concatenate([np.arange(0, 1 << 16, dtype=np.uint64),
                         rng.integers(0, 1 << 31, size=1 << 16, dtype=np.uint64),
                         np.array([(1 << 31) - 1], dtype=np.uint64)])
    for d in list(range(1, 130)) + [256, 1024, 4096, 65536]:
        m = np.uint64(0xFFFFFFFF // d)
        q = (xs * m) >> np.uint64(32)
        q = q + ((q + np.uint64(1)) * np.uint64(d) <= xs).astype(np.uint64)
        assert np.array_equal(q, xs // np.uint64(d)), d
