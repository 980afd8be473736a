"""Build libnlp.so (gfx950) in-tree.

    python neighborhood-link-prediction-openmp_amd/build.py

hipcc cross-compiles for gfx950 without a GPU.  Floating-point flags matter for
parity: no fast-math, no FP contraction, correctly rounded fp32 division (the
reference's scores are IEEE float divisions on x86-64, predict.hxx:542-749).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libnlp.so")
SOURCES = [os.path.join(HERE, "csrc", f) for f in ("nlp.hip",)]


def deps():
    """Every file the library is built from: the sources, every header under
    csrc/ (globbed, so a new header is never missed) and the C-ABI header."""
    import glob
    return SOURCES + sorted(glob.glob(os.path.join(HERE, "csrc", "*.hpp"))) + [os.path.join(ROOT, "include", "nlp.h")]

HIPCC_FLAGS = [
    "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
    "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-fast-math",
    "-Wall", "-Wno-unused-function",
]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    return "hipcc"


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(d) > t for d in deps() if os.path.exists(d))


CPP_TEST_SRC = os.path.join(ROOT, "tests", "cpp", "predict_main.cxx")
CPP_TEST_BIN = os.path.join(HERE, "predict_main")


def build_cpp_test(verbose=True):
    """The C++ drop-in check (tests/cpp/predict_main.cxx) linked against libnlp.so."""
    deps = [CPP_TEST_SRC, LIB, os.path.join(ROOT, "include", "nlp", "predict.hxx")]
    if os.path.exists(CPP_TEST_BIN) and all(os.path.getmtime(d) <= os.path.getmtime(CPP_TEST_BIN) for d in deps):
        return CPP_TEST_BIN
    cmd = ["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"), CPP_TEST_SRC, "-L", HERE, "-lnlp",
           "-Wl,-rpath," + HERE, "-o", CPP_TEST_BIN]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return CPP_TEST_BIN


MAIN_SRC = os.path.join(HERE, "nlp_main.cxx")
MAIN_BIN = os.path.join(HERE, "nlp_main")


def build_main(verbose=True):
    """nlp_main: the main.cxx-style experiment driver (host ingest + sweep) over libnlp.so."""
    deps = [MAIN_SRC, LIB] + [os.path.join(ROOT, "include", "nlp", f) for f in ("predict.hxx", "ingest.hxx")]
    if os.path.exists(MAIN_BIN) and all(os.path.getmtime(d) <= os.path.getmtime(MAIN_BIN) for d in deps):
        return MAIN_BIN
    cmd = ["g++", "-std=c++17", "-O3", "-fopenmp", "-Wall", "-Wno-unknown-pragmas", "-I", os.path.join(ROOT, "include"),
           MAIN_SRC, "-L", HERE,
           "-lnlp", "-Wl,-rpath," + HERE, "-o", MAIN_BIN]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return MAIN_BIN


INGEST_SRC = os.path.join(ROOT, "tests", "cpp", "ingest_dev_main.cxx")
INGEST_BIN = os.path.join(HERE, "ingest_dev_main")


def build_ingest_dev(verbose=True):
    """ingest_dev_main: nlp_main's device ingest route (readMtxPairs + nlp_dcsr_*) for the GPU ingest tests."""
    deps = [INGEST_SRC, LIB] + [os.path.join(ROOT, "include", "nlp", f) for f in ("predict.hxx", "ingest.hxx")]
    if os.path.exists(INGEST_BIN) and all(os.path.getmtime(d) <= os.path.getmtime(INGEST_BIN) for d in deps):
        return INGEST_BIN
    cmd = ["g++", "-std=c++17", "-O2", "-fopenmp", "-I", os.path.join(ROOT, "include"), INGEST_SRC, "-L", HERE,
           "-lnlp", "-Wl,-rpath," + HERE, "-o", INGEST_BIN]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return INGEST_BIN


BENCH_SRC = os.path.join(ROOT, "tests", "cpp", "dropin_bench.cxx")
BENCH_BIN = os.path.join(HERE, "dropin_bench")


def build_dropin_bench(verbose=True):
    """dropin_bench: the drop-in header's cost per call (bench.py's dropin object), OpenMP like main.cxx."""
    deps = [BENCH_SRC, LIB, os.path.join(ROOT, "include", "nlp", "predict.hxx")]
    if os.path.exists(BENCH_BIN) and all(os.path.getmtime(d) <= os.path.getmtime(BENCH_BIN) for d in deps):
        return BENCH_BIN
    cmd = ["g++", "-std=c++17", "-O3", "-fopenmp", "-I", os.path.join(ROOT, "include"), BENCH_SRC, "-L", HERE,
           "-lnlp", "-Wl,-rpath," + HERE, "-o", BENCH_BIN]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return BENCH_BIN


def build(force=False, verbose=True):
    if not force and not needs_build():
        build_cpp_test(verbose)
        build_main(verbose)
        build_dropin_bench(verbose)
        build_ingest_dev(verbose)
        return LIB
    cmd = [hipcc()] + HIPCC_FLAGS + [f for f in os.environ.get("NLP_HIPCC_EXTRA", "").split() if f] + SOURCES + \
        ["-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    build_cpp_test(verbose)
    build_main(verbose)
    build_dropin_bench(verbose)
    build_ingest_dev(verbose)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
