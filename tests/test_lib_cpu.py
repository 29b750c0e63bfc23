"""CPU-side checks of the C-ABI library: it builds for gfx950, loads beside torch's HIP runtime,
exports every entry point include/navenv.h declares, and validates arguments on the host (no
kernel is launched by these calls)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "navenv.h")
LIB = os.path.join(PKG, "nav", "libnavenv.so")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|int64_t|void)\s+(nav_\w+)\s*\(", src, re.M)))


@pytest.fixture(scope="module")
def navlib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-j4", "-C", PKG], check=True)
    from nav import _lib
    return _lib.lib()


def test_header_has_entry_points():
    fns = header_functions()
    assert len(fns) >= 25
    assert {"nav_env_step", "nav_env_reset", "nav_agent_step", "nav_act",
            "nav_mlp_forward", "nav_adam"} <= set(fns)


def test_library_exports_every_declared_symbol(navlib):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\b(nav_\w+)\b", out))
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing
    from nav._lib import SIGNATURES
    bound = {s[0] for s in SIGNATURES}
    assert set(header_functions()) == bound


def test_integration_table_names_the_abi():
    """INTEGRATION.md's entry-point table names every declared entry point, and no name that
    the header does not declare (stale docs)."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    table = doc[doc.index("Entry points and the reference interface"):doc.index("## 3.")]
    named = set(re.findall(r"`(nav_\w+)`", table))
    fns = set(header_functions())
    assert fns - named == set(), sorted(fns - named)
    assert named - fns == set(), sorted(named - fns)


def test_gfx950_code_object_present(navlib):
    # the offload bundle carries a gfx950 code object (and no other GPU target)
    blob = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert not re.search(rb"amdgcn-amd-amdhsa--gfx9[0-4]\d", blob)


def test_abi_and_layout(navlib):
    from nav.mlp import layer_offsets
    from nav._lib import NavMlp
    assert navlib.nav_abi_version() == 11
    assert navlib.nav_demo_index_res() in (1, 2, 4, 8)
    # the CPU port's index (cpu_baseline) is built at the same resolution
    from oracle import oracle as O
    assert O.lib().orc_demo_index_res() == navlib.nav_demo_index_res()
    for d_in, d_out, hidden, nh in ((2, 2, 200, 3), (4, 1, 200, 3), (2, 2, 256, 2),
                                    (4, 1, 256, 2), (4, 1, 32, 1)):
        hp = (hidden + 31) // 32 * 32
        offs, count = layer_offsets(d_in, d_out, hp, nh)
        assert navlib.nav_mlp_param_count(d_in, d_out, hp, nh) == count
        assert navlib.nav_mlp_packed_count(hp, nh) == (nh - 1) * 2 * (hp * hp + hp)
        d = NavMlp(d_in, d_out, hidden, hp, nh, 16, 16)
        for l, (w, b, _, _) in enumerate(offs):
            wo, bo = C.c_int64(), C.c_int64()
            navlib.nav_mlp_layer_offsets(C.byref(d), l, C.byref(wo), C.byref(bo))
            assert (wo.value, bo.value) == (w, b)
    # hidden width must be padded to a multiple of 32 within 256
    from nav._lib import NavError
    with pytest.raises(NavError):
        navlib.nav_mlp_param_count(2, 2, 200, 3)


def test_host_argument_validation(navlib):
    from nav._lib import NavEnvSoa, NavError, params_struct
    p = params_struct()
    assert p.seed_lo == 1707366464 and p.path_length0 == 50 and p.max_action == 5.0
    bad = NavEnvSoa(16, None, None, None, None, None, None, None, None, None)
    with pytest.raises(NavError, match="invalid argument"):
        navlib.nav_env_init(C.byref(p), C.byref(bad), 1, 1, None, None)
    with pytest.raises(NavError, match="invalid argument"):
        navlib.nav_env_step(C.byref(p), C.byref(bad), None, None, None, None)
    with pytest.raises(NavError, match="invalid argument"):
        navlib.nav_grad_reduce(None, None, 1, None, 1, None, None)
    from nav._lib import NavMlp
    d = NavMlp(4, 1, 256, 256, 2, 16, 16)
    with pytest.raises(NavError, match="invalid argument"):  # no masks
        navlib.nav_mlp_wgrad(C.byref(d), 1, 64, 16, 4, 0, None, None,
                             (C.c_void_p * 1)(16), 1, None, (C.c_void_p * 1)(16), 4, None)
    assert navlib.nav_mlp_edge_count(4, 1, 256, 2) == 4 * 256 + 256 + 256 + 256 + 4
    assert navlib.nav_mlp_hidden_count(256, 2) == 256 * 256
    empty = NavEnvSoa(0, None, None, None, None, None, None, None, None, None)
    navlib.nav_env_reset(C.byref(p), C.byref(empty), None, None, None)  # n = 0: no-op
