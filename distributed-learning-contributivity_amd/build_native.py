"""Build libmplc_hip.so (all HIP kernels + the C ABI of include/mplc_hip.h) for gfx950, in-tree.

    python distributed-learning-contributivity_amd/build_native.py [-v] [--force]

Each csrc/*.hip is compiled to an object with hipcc (parallel, timestamp-checked), then linked into
mplc/lib/libmplc_hip.so.  The .so is git-ignored but travels to the GPU box with the gpurun snapshot.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG_ROOT = os.path.dirname(os.path.abspath(__file__))
REPO_ROOT = os.path.dirname(PKG_ROOT)
CSRC = os.path.join(PKG_ROOT, "csrc")
INCLUDE = os.path.join(REPO_ROOT, "include")
BUILD = os.path.join(PKG_ROOT, "build")
LIB_DIR = os.path.join(PKG_ROOT, "mplc", "lib")
LIB = os.path.join(LIB_DIR, "libmplc_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# -ffp-contract=on: multiply-adds fuse only within one source expression, as the source writes them (hipcc's default
# also lets the backend fuse across statements, and which product it picks can move with unrelated code: a refactor of
# dense1_bwd_adam_kernel flipped Adam's fusion, profiles/r06_adam_contraction.txt); `#pragma clang fp contract(off)`
# still marks the code whose every operation rounds on its own (Adam, RMSprop, FedAvg)
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
          "-Wno-unused-result", "-munsafe-fp-atomics", "-ffp-contract=on"]


def _deps(src):
    hdrs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return [src] + hdrs


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


# Per-source extra flags.  mnist_cnn.hip: no SLP vectorisation - packed f32 VALU (v_pk_add_f32 and the v_mov
# shuffles that feed it) issued beside f32 MFMAs costs more issue cycles than the scalar ops it replaces
# (MI355X_MICROARCH.md, per-instruction cycle constants), and it hoisted the Winograd V arithmetic of the
# software-pipelined conv k-loops out of the MFMA gaps.  cifar_cnn.hip likewise (its Winograd loops: 10-25 % fewer
# VALU instructions; every VALU instruction costs an f32 MFMA stream 2.5-3.5 cycles); its two head
# kernels live in cifar_head.hip with the default flags, which keeps their expf / logf / dot-product code as it was.
FILE_FLAGS = {"mnist_cnn.hip": ["-fno-slp-vectorize"], "mnist_wgrad.hip": ["-fno-slp-vectorize"],
              "cifar_cnn.hip": ["-fno-slp-vectorize"]}


def _compile(src, obj, verbose):
    cmd = [HIPCC] + CFLAGS + FILE_FLAGS.get(os.path.basename(src), []) + ["-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {os.path.basename(src)}:\n{r.stdout}\n{r.stderr}")
    if verbose and r.stderr.strip():
        print(r.stderr, flush=True)
    return obj


# Host-side AddressSanitizer + UndefinedBehaviorSanitizer build: the C ABI's argument validation,
# workspace sizing and launch set-up run instrumented; device code is compiled as usual (GPU sanitizers are not
# available on the pool).  Each -fsanitize= sits directly after -Xarch_host so that it applies to the host pass
# only.  Output: build/asan/libmplc_hip.so (never the product library).
SAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
             "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=undefined"]
SAN_BUILD = os.path.join(BUILD, "asan")
SAN_LIB = os.path.join(SAN_BUILD, "libmplc_hip.so")


def build(verbose=False, force=False, jobs=8, sanitize=False):
    global CFLAGS
    build_dir = SAN_BUILD if sanitize else BUILD
    lib = SAN_LIB if sanitize else LIB
    os.makedirs(build_dir, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    if not srcs:
        raise RuntimeError("no HIP sources found")
    base = CFLAGS
    if sanitize:
        CFLAGS = CFLAGS + SAN_FLAGS
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(build_dir, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if force or _stale(o, _deps(s)):
            todo.append((s, o))
    try:
        if todo:
            with cf.ThreadPoolExecutor(max_workers=min(jobs, len(todo))) as ex:
                list(ex.map(lambda so: _compile(so[0], so[1], verbose), todo))
    finally:
        CFLAGS = base
    if force or todo or _stale(lib, objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", lib] + objs
        if sanitize:
            cmd += ["-fsanitize=address", "-fsanitize=undefined", "-shared-libsan"]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return lib


# Alternate kernel forms kept in the source because they are bit-identical to the product kernels (the matrix core
# accumulates as an fma chain) and win at other batch sizes: the MFMA form of MNIST's dense1_bwd_adam
# (MPLC_D1_MFMA=1), the VALU form of CIFAR's dense5_bwd (MPLC_D5_MFMA=0), the 32-row form of its dense5_fwd at
# every batch size (MPLC_D5F16_MAX=0) and conv4_fwd's remainder group as a padded 16-tile MFMA group instead of
# 4x4x1 MFMAs (MPLC_WINO_QUAD=0).  build() links them into one variant
# library, mplc/lib/variants/libmplc_hip_alt.so, which tests/test_variants_gpu.py runs against the product library
# (bit-identical models), so the non-default bodies cannot rot unseen.
VARIANTS = {"alt": {"mnist_cnn.hip": ["-DMPLC_D1_MFMA=1"], "cifar_cnn.hip": ["-DMPLC_D5_MFMA=0", "-DMPLC_D5F16_MAX=0",
                                                                         "-DMPLC_WINO_QUAD=0"]}}
VARIANT_DIR = os.path.join(LIB_DIR, "variants")


def build_variants(verbose=False, force=False, jobs=8):
    """Variant libraries (VARIANTS): the listed sources recompiled with their flags, linked with the product objects
    of every other source.  Call after build()."""
    os.makedirs(VARIANT_DIR, exist_ok=True)
    out = []
    for name, flags in VARIANTS.items():
        vdir = os.path.join(BUILD, "variant_" + name)
        os.makedirs(vdir, exist_ok=True)
        objs, todo = [], []
        for src in sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
            base = os.path.basename(src)
            if base in flags:
                o = os.path.join(vdir, base[:-4] + ".o")
                flag_file = o + ".flags"
                stale = force or _stale(o, _deps(src)) or not os.path.exists(flag_file) or \
                    open(flag_file).read() != " ".join(flags[base])
                if stale:
                    todo.append((src, o, flags[base], flag_file))
            else:
                o = os.path.join(BUILD, base[:-4] + ".o")
            objs.append(o)

        def comp(item):
            src, o, fl, ff = item
            cmd = [HIPCC] + CFLAGS + FILE_FLAGS.get(os.path.basename(src), []) + fl + ["-c", src, "-o", o]
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed for variant {name} {os.path.basename(src)}:\n{r.stderr}")
            with open(ff, "w") as f:
                f.write(" ".join(fl))
        if todo:
            with cf.ThreadPoolExecutor(max_workers=min(jobs, len(todo))) as ex:
                list(ex.map(comp, todo))
        lib = os.path.join(VARIANT_DIR, f"libmplc_hip_{name}.so")
        if force or todo or _stale(lib, objs):
            cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", lib] + objs
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"link failed for variant {name}:\n{r.stderr}")
        out.append(lib)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--sanitize", action="store_true", help="host ASan/UBSan build into build/asan/")
    a = ap.parse_args()
    print(build(verbose=a.verbose, force=a.force, sanitize=a.sanitize))
    if not a.sanitize:
        print("\n".join(build_variants(verbose=a.verbose, force=a.force)))
    sys.exit(0)
