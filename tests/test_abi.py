"""CPU-side checks of the C-ABI library (no kernel launches): it loads, exports every symbol that
include/cfm_encoder.h declares, and its host helpers agree with the oracle."""
import ctypes
import os
import re

import numpy as np
import pytest

import conformer_oracle as O
from conftest import ROOT


def _declared_symbols(header="cfm_encoder.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cfm_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_header_symbols():
    from conformer_amd import _lib
    lib = _lib.load()
    declared = _declared_symbols()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(_lib.EXPORTED_SYMBOLS)
    # and the .so really defines them (not just resolvable through another library)
    out = os.popen(f"nm -D --defined-only {_lib.LIB_PATH}").read()
    for name in declared:
        assert re.search(rf"\bT {name}\b", out), name
    ctc = _declared_symbols("cfm_ctc.h")
    assert set(ctc) == set(_lib.CTC_SYMBOLS)
    train = _declared_symbols("cfm_train.h")
    assert set(train) == set(_lib.TRAIN_SYMBOLS)
    joint = _declared_symbols("cfm_joint.h")
    assert set(joint) == set(_lib.JOINT_SYMBOLS)
    stream = _declared_symbols("cfm_stream.h")
    assert set(stream) == set(_lib.STREAM_SYMBOLS)
    mel = _declared_symbols("cfm_mel.h")
    assert set(mel) == set(_lib.MEL_SYMBOLS)
    rl = _declared_symbols("cfm_rnnt_loss.h")
    assert set(rl) == set(_lib.RNNT_LOSS_SYMBOLS)
    aug = _declared_symbols("cfm_augment.h")
    assert set(aug) == set(_lib.AUGMENT_SYMBOLS)
    dec = _declared_symbols("cfm_rnnt_decode.h")
    assert set(dec) == set(_lib.RNNT_DECODE_SYMBOLS)
    comm = _declared_symbols("cfm_comm.h")
    assert set(comm) == set(_lib.COMM_SYMBOLS)
    cs = _declared_symbols("cfm_cache_stream.h")
    assert set(cs) == set(_lib.CACHE_STREAM_SYMBOLS)
    from conformer_amd import cache_stream
    assert set(cache_stream.SYMBOLS) == set(cs)
    for name in ctc + train + joint + stream + mel + rl + aug + dec + comm + cs:
        assert hasattr(lib, name) and re.search(rf"\bT {name}\b", out), name


def test_fp16_build_exports_the_same_abi():
    """libcfm_f16.so (the fp16 compute mode) is the same sources with the other 16-bit format: the same
    exported symbols, and each build accepts only its own 16-bit mode (checked before any GPU call)."""
    from conformer_amd import _lib, make_cfg
    lib16 = _lib.load("fp16")
    lib = _lib.load()
    assert lib.cfm_half_mode() == _lib.CFM_COMPUTE_BF16 and lib16.cfm_half_mode() == _lib.CFM_COMPUTE_FP16
    out = os.popen(f"nm -D --defined-only {_lib.LIB16_PATH}").read()
    ref = os.popen(f"nm -D --defined-only {_lib.LIB_PATH}").read()
    syms = lambda t: sorted(set(re.findall(r"\bT (cfm_[a-z0-9_]+)\b", t)))   # noqa: E731
    assert syms(out) == syms(ref) and len(syms(out)) > 100
    h = ctypes.c_void_p()
    cfg = make_cfg(80, 2, 64, n_heads=4)
    assert lib.cfm_encoder_create(ctypes.byref(cfg), 0, _lib.CFM_COMPUTE_FP16, ctypes.byref(h)) == 2
    assert b"libcfm_f16" in lib.cfm_last_error()
    assert lib16.cfm_encoder_create(ctypes.byref(cfg), 0, _lib.CFM_COMPUTE_BF16, ctypes.byref(h)) == 2
    assert b"libcfm.so" in lib16.cfm_last_error()


def test_encoded_length_matches_oracle():
    from conformer_amd import _lib
    lib = _lib.load()
    Ls = np.arange(0, 5001)
    ref = O.calc_length(Ls)
    got = np.array([lib.cfm_encoded_length(int(L)) for L in Ls])
    np.testing.assert_array_equal(got, ref)


def test_create_without_gpu_fails_cleanly():
    """Without a GPU the library must report an error status, never crash or fall back."""
    import torch
    if torch.cuda.is_available():
        return
    from conformer_amd import _lib, make_cfg
    lib = _lib.load()
    h = ctypes.c_void_p()
    cfg = make_cfg(80, 2, 64, n_heads=4)
    st = lib.cfm_encoder_create(ctypes.byref(cfg), 0, 1, ctypes.byref(h))
    assert st != 0
    assert lib.cfm_last_error()


def test_bad_config_rejected():
    from conformer_amd import _lib, make_cfg
    lib = _lib.load()
    h = ctypes.c_void_p()
    cfg = make_cfg(80, 2, 60, n_heads=7)        # d_model % n_heads != 0
    assert lib.cfm_encoder_create(ctypes.byref(cfg), 0, 1, ctypes.byref(h)) == 1
    cfg = make_cfg(80, 2, 64, n_heads=4, subsampling_factor=8)
    assert lib.cfm_encoder_create(ctypes.byref(cfg), 0, 1, ctypes.byref(h)) == 2


def test_c_consumer(tmp_path):
    """The headers compile as plain C99 (-pedantic) and a C program links libcfm.so and gets status
    codes and messages back on the host (tests/c/abi_smoke.c): the boundary needs no C++ or torch."""
    import shutil
    import subprocess
    from conformer_amd import _lib
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("gcc not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    libdir = os.path.dirname(_lib.LIB_PATH)
    exe = str(tmp_path / "abi_smoke")
    subprocess.run([gcc, "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I", os.path.join(root, "include"),
                    os.path.join(root, "tests", "c", "abi_smoke.c"), "-L", libdir, "-lcfm", f"-Wl,-rpath,{libdir}",
                    "-o", exe], check=True, capture_output=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("ok:") == 5
