"""CPU reproduction of the deadlock behind round 4's two-rank hang.

threadpoolctl (used by sklearn and by tau_init._numpy_blas) finds the loaded BLAS /
OpenMP libraries with ``dl_iterate_phdr`` and a ctypes callback written in Python:
glibc holds the loader's lock while the callback runs, and the callback needs the GIL.
A thread that holds the GIL and loads a library -- here a ``ctypes.PyDLL`` call that
dlopens (libpert_hip's launch entry points are bound through PyDLL, and the HIP runtime
dlopens lazily), in general any extension-module import -- waits for the loader's lock
with the GIL in hand.  Neither thread moves again.

Run: ``python tools/dl_deadlock_repro.py``.  Without the fix the script stops itself
through faulthandler after 20 s and prints both stacks (the scanner inside threadpoolctl's
callback, the main thread inside the PyDLL call); ``--prepared`` makes the scan once on
the main thread first, as tau_init.prepare_host_threads() does, and the helper then
reuses the controller (no scan): it finishes.
"""
import ctypes
import faulthandler
import glob
import os
import subprocess
import sys
import tempfile
import threading
import time

SRC = r'''
#include <dlfcn.h>
int do_dlopen(const char* p){ void* h = dlopen(p, RTLD_NOW|RTLD_LOCAL); if(!h) return 1; dlclose(h); return 0; }
'''


def main(prepared: bool):
    faulthandler.dump_traceback_later(20, exit=True)
    d = tempfile.mkdtemp()
    c, so = os.path.join(d, "dl.c"), os.path.join(d, "libdl_repro.so")
    open(c, "w").write(SRC)
    subprocess.check_call(["gcc", "-shared", "-fPIC", "-O2", c, "-o", so, "-ldl"])
    from threadpoolctl import ThreadpoolController
    lib = ctypes.PyDLL(so)                               # the call keeps the GIL
    lib.do_dlopen.argtypes = [ctypes.c_char_p]
    cands = [p for p in glob.glob("/usr/lib/x86_64-linux-gnu/lib*.so*")
             if not any(w in os.path.basename(p) for w in ("python", "san.", "san_", "memusage", "pcprofile"))][:400]
    ctl = ThreadpoolController() if prepared else None   # the scan, made here once
    stop = []

    def scanner():
        n = 0
        while not stop:
            (ctl.info() if ctl is not None else ThreadpoolController().info())
            n += 1
        print("helper: {} controller uses".format(n))
    t = threading.Thread(target=scanner)
    t.start()
    t0 = time.time()
    for p in cands:
        lib.do_dlopen(p.encode())
    stop.append(1)
    t.join()
    print("no deadlock: {} dlopens under the GIL in {:.2f} s".format(len(cands), time.time() - t0))


if __name__ == "__main__":
    main("--prepared" in sys.argv)
