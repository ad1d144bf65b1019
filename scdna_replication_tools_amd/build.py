"""Build libpert_hip.so in-tree for gfx950 (hipcc, no JIT cache).

    python -m scdna_replication_tools_amd.build [--force] [--verbose]

Provenance: the SHA-256 of the sources the library is compiled from (``SOURCES`` +
headers, ``source_hash()``) is baked into the binary and returned by
``pert_version()`` ("... src=<hash>").  ``build()`` rebuilds whenever the library's
embedded hash differs from the tree's (not by file times), and ``_native.lib()``
refuses a library whose hash does not match the sources next to it, so a stale
binary shipped with the tree fails loudly instead of passing tests.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SOURCES = [os.path.join(HERE, "csrc", "pert_kernels.hip"), os.path.join(HERE, "csrc", "tau_kernels.hip"),
           os.path.join(HERE, "csrc", "pert_comm.hip")]
DEPS = SOURCES + [os.path.join(HERE, "csrc", "pert_math.h"), os.path.join(ROOT, "include", "pert_hip.h")]
OUT = os.path.join(HERE, "libpert_hip.so")
OBJ_DIR = os.path.join(HERE, "build_obj")
ARCH = os.environ.get("PERT_OFFLOAD_ARCH", "gfx950")
HASH_LEN = 16
FLAGS = ["-fno-slp-vectorize", "-fno-signed-zeros"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def source_hash() -> str:
    """SHA-256 (first 16 hex digits) over the library's sources, in a fixed order."""
    h = hashlib.sha256()
    for d in DEPS:
        h.update(os.path.basename(d).encode())
        with open(d, "rb") as fh:
            h.update(fh.read())
    h.update(ARCH.encode())
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()[:HASH_LEN]


def embedded_hash(path: str = OUT):
    """The source hash baked into a built library (read from its bytes; no load)."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as fh:
        m = re.search(rb"pert_hip [0-9.]+ gfx950 src=([0-9a-f]{%d})" % HASH_LEN, fh.read())
    return m.group(1).decode() if m else None


def up_to_date() -> bool:
    return embedded_hash(OUT) == source_hash()


def _object_hash(src: str) -> str:
    """Hash of one translation unit's inputs: the source, the shared headers, arch and flags."""
    h = hashlib.sha256()
    for d in [src] + DEPS[len(SOURCES):]:
        with open(d, "rb") as fh:
            h.update(fh.read())
    h.update(ARCH.encode())
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()[:HASH_LEN]


def _run(cmd, what, verbose=False):
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout + res.stderr)
        raise RuntimeError("hipcc failed building {}".format(what))
    if verbose:
        sys.stderr.write(res.stderr)


def build(force: bool = False, verbose: bool = False) -> str:
    """Each source is compiled to its own object (kept beside OUT, named by the hash of its
    inputs, so an unchanged source is not recompiled); pert_version() with the whole tree's
    source_hash() is a one-line object of its own; then one link."""
    if not force and up_to_date():
        return OUT
    # -fno-slp-vectorize: SLP packs independent fp32 chains into v_pk_* pairs whose register
    # pairing and shuffles cost 50-70 VGPRs in the enumerated passes (occupancy), for no gain
    base = [hipcc(), "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", *FLAGS, "-I" + os.path.join(ROOT, "include")]
    objs = []
    for src in SOURCES:
        obj = os.path.join(OBJ_DIR, "{}.{}.o".format(os.path.splitext(os.path.basename(src))[0], _object_hash(src)))
        if force or not os.path.exists(obj):
            os.makedirs(OBJ_DIR, exist_ok=True)
            cmd = base + ["-c", src, "-o", obj + ".tmp"]
            if verbose:
                cmd.append("-Rpass-analysis=kernel-resource-usage")
            _run(cmd, obj, verbose)
            os.replace(obj + ".tmp", obj)
        objs.append(obj)
    ver = os.path.join(OBJ_DIR, "pert_version.c")
    os.makedirs(OBJ_DIR, exist_ok=True)
    with open(ver, "w") as fh:
        # "src=<hash>": the sources this binary was compiled from (_native.lib() refuses a
        # library whose hash differs from its tree)
        fh.write('const char* pert_version(void) {{ return "pert_hip 0.2 {} src={}"; }}\n'.format(ARCH, source_hash()))
    _run([os.environ.get("CC", "gcc"), "-O2", "-fPIC", "-c", ver, "-o", ver[:-2] + ".o"], ver, verbose)
    _run([hipcc(), "--offload-arch=" + ARCH, "-shared", "-fPIC", *objs, ver[:-2] + ".o", "-o", OUT + ".tmp"], OUT,
         verbose)
    for f in os.listdir(OBJ_DIR):                       # objects of older sources
        if f.endswith(".o") and os.path.join(OBJ_DIR, f) not in objs and f != "pert_version.o":
            os.remove(os.path.join(OBJ_DIR, f))
    os.replace(OUT + ".tmp", OUT)
    return OUT


HOST_SOURCES = [os.path.join(HERE, "csrc", "pert_host.c")]
HOST_OUT = os.path.join(HERE, "libpert_host.so")
# no contraction into fma, no reassociation: the helper repeats numpy's fp32 operations exactly
HOST_FLAGS = ["-O2", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math", "-std=c99"]


def host_source_hash() -> str:
    h = hashlib.sha256()
    for d in HOST_SOURCES:
        with open(d, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(HOST_FLAGS).encode())
    return h.hexdigest()[:HASH_LEN]


def host_embedded_hash(path: str = HOST_OUT):
    """The source hash baked into libpert_host.so (``pert_host_version()``, read from its bytes)."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as fh:
        m = re.search(rb"pert_host src=([0-9a-f]{%d})" % HASH_LEN, fh.read())
    return m.group(1).decode() if m else None


def build_host(force: bool = False) -> str:
    """libpert_host.so (gcc): the CPU helpers of tau_init's exact path.  The hash of its
    sources is compiled into it (``pert_host_version()``); it is rebuilt when that differs
    from the tree's, and tau_init refuses a library whose hash does not match."""
    want = host_source_hash()
    if not force and host_embedded_hash() == want:
        return HOST_OUT
    cmd = [os.environ.get("CC", "gcc"), *HOST_FLAGS, '-DPERT_HOST_SRC="{}"'.format(want), *HOST_SOURCES,
           "-o", HOST_OUT + ".tmp"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout + res.stderr)
        raise RuntimeError("gcc failed building {}".format(HOST_OUT))
    os.replace(HOST_OUT + ".tmp", HOST_OUT)
    stale = HOST_OUT + ".src"                     # the stamp file of earlier builds
    if os.path.exists(stale):
        os.remove(stale)
    return HOST_OUT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, verbose=a.verbose))
    print(build_host(force=a.force))


if __name__ == "__main__":
    main()
