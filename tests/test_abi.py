"""The C-ABI library: builds, loads, exports every symbol include/*.h
declares, and fails loudly (no CPU fallback) without a gfx950 device."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

from babble_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(bv_[a-z0-9_]+)\s*\(", src):
            names.add(m.group(1))
    return names


def test_header_declares_what_we_bind():
    assert declared_functions() == set(native.EXPORTS)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = declared_functions() - exported
    assert not missing, missing


def test_abi_version_and_code_object():
    L = native.lib()
    assert L.bv_abi_version() == native.ABI_VERSION == 2
    # the library carries gfx950 device code (offload bundle entry name)
    blob = open(native.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_create_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    ctx = ctypes.c_void_p()
    rc = native.lib().bv_create(ctypes.byref(ctx), 0, 0)
    assert rc == native.BV_E_NODEVICE and not ctx.value


def test_null_args():
    L = native.lib()
    assert L.bv_verify_batch(None, None, None) == native.BV_E_ARGS
    assert L.bv_verify_batch_device(None, None, None, None, 0) == native.BV_E_ARGS
    assert L.bv_sha256_batch(None, 0, None, None, None) == native.BV_E_ARGS
    assert L.bv_get_timing(None, None) == native.BV_E_ARGS
