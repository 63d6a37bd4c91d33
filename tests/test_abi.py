"""The C ABI library loads, exports every entry point of include/marlsched.h,
and validates configurations (no device needed)."""
import ctypes as ct
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    with open(os.path.join(REPO, "include", "marlsched.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(ms_[a-z0-9_]+)\s*\(", src)) - {"ms_env"})


def test_exports_every_declared_symbol(ms):
    declared = _declared()
    assert declared == sorted(ms._lib.EXPORTED)
    L = ct.CDLL(ms.LIB_PATH)
    for name in declared:
        assert hasattr(L, name), name


def test_config_shape_and_validation(ms):
    abi = ms.abi
    cfg = abi.named_config("cfg3")
    sh = abi.MsShape()
    ms.check(ms.lib.ms_config_shape(ct.byref(cfg), ct.byref(sh)))
    py = abi.config_shape(cfg)
    assert (sh.max_offers, sh.acc_obs_dim, sh.acc_obs_stride, sh.off_obs_dim, sh.off_obs_stride) == (
        24, 51, 52, 18, 20)
    assert sh.acc_obs_dim == py["acc_obs_dim"] and sh.price_actions == py["price_actions"] == 13
    bad = abi.make_config(2, 2, 2, **abi.README_JOBS)
    bad.n_fix_prices = 1  # fewer fixed prices than job kinds
    with pytest.raises(ms.MarlSchedError):
        ms.check(ms.lib.ms_config_shape(ct.byref(bad), ct.byref(sh)))
    assert b"fixed prices" in ms.lib.ms_last_error()
    big = abi.make_config(64, 4, 2, **abi.README_JOBS)  # O = 128 > 126
    with pytest.raises(ms.MarlSchedError):
        ms.check(ms.lib.ms_config_shape(ct.byref(big), ct.byref(sh)))


def test_named_configs_shapes(ms):
    abi = ms.abi
    for name, (d_acc, a_acc, d_off, a_off) in dict(cfg1=(11, 5, 6, 3), cfg2=(27, 13, 10, 5), cfg3=(51, 25, 18, 9),
                                                    cfg4=(99, 49, 34, 17), cfg5=(195, 97, 66, 33)).items():
        s = abi.config_shape(abi.named_config(name))  # SURVEY.md §8 shape table
        assert (s["acc_obs_dim"], s["acc_actions"], s["off_obs_dim"], s["off_actions"]) == (d_acc, a_acc, d_off, a_off)
