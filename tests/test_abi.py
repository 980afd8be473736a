"""CPU-side checks of the drop-in boundary: libnlp.so builds for gfx950, loads,
and exports every symbol include/nlp.h declares; the C++ mirror header
compiles.  No compute calls (there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nlp.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nlp_[a-z_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    f = declared_functions()
    for name in ("nlp_graph_create", "nlp_predict", "nlp_graph_destroy", "nlp_status_string",
                 "nlp_predict_device", "nlp_select_edges_device"):
        assert name in f


def test_library_exports_every_declared_symbol(nlp):
    L = nlp.lib()
    missing = [f for f in declared_functions() if not hasattr(L, f)]
    assert not missing, missing
    assert set(nlp.EXPORTS) <= set(declared_functions())


def test_library_has_gfx950_code_object(nlp):
    nlp.lib()
    data = open(nlp.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_status_and_metric_strings(nlp):
    L = nlp.lib()
    assert L.nlp_status_string(0) == b"ok"
    assert L.nlp_status_string(4) == b"no gfx950 device"
    assert L.nlp_metric_name(1) == b"JaccardCoefficient"
    assert L.nlp_metric_name(8) == b"ResourceAllocationScore"
    assert L.nlp_version() >= 100


def test_invalid_arguments_rejected_without_device(nlp):
    L = nlp.lib()
    h = ctypes.c_void_p()
    assert L.nlp_graph_create(None, None, 0, 0, ctypes.byref(h)) == 1
    cnt = ctypes.c_uint64()
    assert L.nlp_predict(None, 0, 4, 0.0, 10, 1, None, ctypes.byref(cnt), None) == 1
    # the asynchronous pair: no handle, nothing pending
    assert L.nlp_predict_device_async(None, 1, 4, 0, 0.0, 10, 0, 2**64 - 1, None, None) == 1
    assert L.nlp_sync(None, ctypes.byref(cnt), None) == 1
    assert L.nlp_status_string(6) == b"an asynchronous prediction needs a synchronous redo"


def test_no_silent_cpu_fallback(nlp):
    """Without a GPU the product path must fail loudly (status NODEVICE), never compute."""
    import numpy as np
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(nlp.NlpError) as e:
        nlp.Graph(np.array([0, 1, 2], np.uint64), np.array([1, 0], np.uint32))
    assert e.value.status == 4


def test_cpp_header_compiles(tmp_path):
    """include/nlp/predict.hxx (the reference-API mirror) compiles with g++ -std=c++17."""
    hdr = os.path.join(ROOT, "include", "nlp", "predict.hxx")
    if not os.path.exists(hdr):
        pytest.skip("C++ mirror header not present")
    src = tmp_path / "t.cxx"
    src.write_text('#include "nlp/predict.hxx"\nint main(){return 0;}\n')
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(src)],
                   check=True)


def test_every_included_header_is_a_build_dependency(nlp):
    """build.py's dependency list covers every header nlp.hip includes (a stale
    libnlp.so after a header-only edit would travel to the GPU box): touching
    any of them makes needs_build() true."""
    from nlp_amd import build as b
    src = open(os.path.join(os.path.dirname(b.__file__), "csrc", "nlp.hip")).read()
    included = re.findall(r'#include\s+"([^"]+\.hpp)"', src)
    deps = {os.path.basename(d) for d in b.deps()}
    assert included and set(included) <= deps, set(included) - deps
    b.build(verbose=False)
    assert not b.needs_build()
    for h in included:
        path = os.path.join(os.path.dirname(b.__file__), "csrc", h)
        st = os.stat(path)
        lib_t = os.path.getmtime(b.LIB)
        try:
            os.utime(path, (st.st_atime, lib_t + 10))
            assert b.needs_build(), h
        finally:
            os.utime(path, (st.st_atime, st.st_mtime))
    assert not b.needs_build()


def test_reference_main_compiles_against_the_dropin_header(tmp_path):
    """The reference's own main.cxx, unmodified, compiled with inc/predict.hxx
    swapped for include/nlp/predict.hxx (oracle/Makefile _ref/main_dropin,
    main.sh:29-42's macros) and linked to libnlp.so: it loads and ingests an
    MTX with the reference's code, and without a GPU its first prediction
    fails loudly with the library's NODEVICE status (no CPU fallback)."""
    if not os.path.exists("/root/reference/main.cxx"):
        pytest.skip("reference not present (GPU box): the prebuilt binary is run by tests/test_gpu_dropin.py")
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present: tests/test_gpu_dropin.py runs it")
    except ImportError:
        pass
    import sys
    from nlp_amd import build as b
    b.build(verbose=False)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_ref/main_dropin"], check=True)
    exe = os.path.join(ROOT, "oracle", "_ref", "main_dropin")
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_golden import chung_lu_mtx
    mtx = str(tmp_path / "g.mtx")
    chung_lu_mtx(mtx, 300, 1200, 0.6, 1)
    r = subprocess.run([exe, mtx, "0", "0"], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "nlp_graph_create: no gfx950 device" in r.stderr
    syms = subprocess.run(["nm", "-D", exe], capture_output=True, text=True).stdout
    assert "nlp_predict_ex" in syms and "nlp_graph_create" in syms
