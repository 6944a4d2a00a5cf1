"""The C-ABI library loads on a GPU-less host and exports every symbol include/bshot_abi.h declares."""
import ctypes
import os
import re

import bshot_py

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "bshot_abi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(bshot_[a-z0-9_]+)\s*\(", src)))


def test_all_declared_symbols_exported():
    L = bshot_py.lib()
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert set(bshot_py.ABI_SYMBOLS) <= set(declared_symbols())


def test_default_params_match_reference_constants():
    p = bshot_py.default_params()
    assert p.seg_radius == 3000.0 and p.seg_max_nn == 300 and p.num_keypoints == 600
    assert p.iss_salient == 60.0 and p.iss_nonmax == 40.0 and p.iss_min_nn == 5
    assert abs(p.iss_gamma21 - 0.975) < 1e-15 and abs(p.iss_gamma32 - 0.975) < 1e-15
    assert p.normal_radius == 3000.0 and p.normal_max_nn == 300 and p.shot_radius == 3000.0
    assert p.map_range == 100000.0 and p.ransac_max_iter == 2000 and p.ransac_thresh == 1500.0
    assert p.icp_max_iter == 10 and p.run_icp == 1


def test_no_gpu_context_fails_loudly_or_works():
    # On a GPU-less host bshot_create must return an error (no silent CPU fallback).
    h = ctypes.c_void_p()
    rc = bshot_py.lib().bshot_create(ctypes.byref(h), 0, None)
    if rc == 0:
        bshot_py.lib().bshot_destroy(h)
    else:
        assert rc < 0


def test_preprocessor_defaults_match_reference():
    p = bshot_py.PreParams()
    bshot_py.lib().bshot_pre_default_params(ctypes.byref(p))
    # src/preprocess.cpp:5-7, include/preprocess.h:43
    assert p.vert_init == -0.6 and p.lowpt_th == -2000.0 and p.have_sel_list == 0 and p.save_sel == 1
    assert bshot_py.LASER_DTYPE.itemsize == 32 and bshot_py.CELL_DTYPE.itemsize == 32
