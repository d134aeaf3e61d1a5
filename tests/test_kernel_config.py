"""The generated kernels' tunables as one frozen KernelConfig (exec/kernel_config.py): built
from defaults, HS_JIT_* and spark.hyperspace.mi.kernel.*, bound into the generators' module
constants, and switched only through ``use`` (restored afterwards)."""
import dataclasses

import pytest

from hyperspace_amd.exec import jit, jit_runs, kernel_config
from hyperspace_amd.exec.kernel_config import KernelConfig


def test_defaults_env_and_conf_layering():
    d = KernelConfig()
    assert d.mj_grid == 8192 and d.rs_bits and not d.mj_key16
    e = KernelConfig.from_env({"HS_JIT_MJ_GRID": "4096", "HS_JIT_RS_BITS": "0",
                               "HS_JIT_UNRELATED": "1"})
    assert e.mj_grid == 4096 and not e.rs_bits and e.scan_vec == d.scan_vec
    c = e.with_conf({"spark.hyperspace.mi.kernel.mj_grid": "2048",
                     "spark.hyperspace.mi.kernel.mj_key16": "true"})
    assert c.mj_grid == 2048 and c.mj_key16 and not c.rs_bits
    with pytest.raises(dataclasses.FrozenInstanceError):
        c.mj_grid = 1


def test_use_binds_module_constants_and_restores():
    before = kernel_config.active()
    shape0 = jit_runs.tags2_shape.__code__   # generator reads RT2_UNROLL at call time
    with kernel_config.use(mj_lds_keys=32, rt2_unroll=2, rs_bits=False) as cfg:
        assert kernel_config.active() is cfg
        assert jit.MJ_LDS_KEYS == 32 and jit_runs.RT2_UNROLL == 2 and not jit_runs.RS_BITS
        with kernel_config.use(mj_lds_keys=16):
            assert jit.MJ_LDS_KEYS == 16 and jit_runs.RT2_UNROLL == 2
        assert jit.MJ_LDS_KEYS == 32
    assert kernel_config.active() is before
    assert jit.MJ_LDS_KEYS == before.mj_lds_keys and jit_runs.RS_BITS == before.rs_bits
    assert shape0 is jit_runs.tags2_shape.__code__


def test_every_field_is_bound_somewhere():
    names = set(jit.__dict__) | set(jit_runs.__dict__)
    missing = [f.name for f in dataclasses.fields(KernelConfig) if f.name.upper() not in names]
    assert not missing, missing


def test_generators_read_no_environment():
    import inspect
    for mod in (jit, jit_runs):
        src = inspect.getsource(mod)
        assert src.count('os.environ.get("HS_JIT_') <= 3, mod.__name__   # cache / dump / record
