"""Which libraries a fit loads, and from where (the two-rank hang).

Runs ``run_pert_model`` on the two-rank API test's tables in a child process with
``LD_DEBUG=files`` (the loader reports every library it maps, on stderr) and markers
written to the same stream around every libpert_hip entry point (bound through PyDLL:
the GIL is held for the call) and every threadpoolctl library scan.  The parent lists each
library loaded after the fit started with the calls in progress at that moment: a load
inside a PyDLL call while a scan runs on another thread is the deadlock of
tools/dl_deadlock_repro.py.

    python tools/dl_probe.py [--world2]   (GPU; --world2: two gloo ranks on one GPU)
"""
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(rank=0, world=1, port=0):
    sys.path.insert(0, ROOT)
    import threading
    import torch
    import threadpoolctl
    from scdna_replication_tools_amd import _native as nat

    def mark(s):
        os.write(2, ("@@{} {} {:.6f} {}\n".format(rank, threading.current_thread().name, time.time(), s)).encode())

    h = nat.lib()
    for name in nat.EXPORTED_SYMBOLS:
        f = getattr(h, name)

        def wrap(*a, _f=f, _n=name):
            mark("ENTER " + _n)
            try:
                return _f(*a)
            finally:
                mark("EXIT " + _n)
        wrap.argtypes, wrap.restype = f.argtypes, f.restype
        setattr(h, name, wrap)
    real = threadpoolctl.ThreadpoolController._find_libraries_with_dl_iterate_phdr

    def scan(self):
        mark("ENTER scan")
        try:
            return real(self)
        finally:
            mark("EXIT scan")
    threadpoolctl.ThreadpoolController._find_libraries_with_dl_iterate_phdr = scan
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{}".format(port), rank=rank, world_size=world)
    from tests.test_gpu_zz_api_ranks import _fit
    mark("FIT_START")
    _fit(device="cuda:0", log_steps=False)
    mark("FIT_END")


def parse(text):
    active = {}          # (rank, thread) -> call in progress
    started = False
    rows = []
    for line in text.splitlines():
        m = re.match(r"@@(\d+) (\S+) ([\d.]+) (\w+) ?(\S*)", line)
        if m:
            rank, thr, _, what, name = m.groups()
            if what == "FIT_START":
                started = True
            elif what == "ENTER":
                active[(rank, thr)] = name
            elif what == "EXIT":
                active.pop((rank, thr), None)
            continue
        f = re.search(r"file=(\S+) \[0\];\s+dynamically loaded by (\S+)", line)
        if f and started:
            rows.append((f.group(1), f.group(2), dict(active)))
    return rows


def main():
    world = 2 if "--world2" in sys.argv else 1
    env = dict(os.environ, LD_DEBUG="files")
    if world == 1:
        cmd = [[sys.executable, __file__, "--child", "0", "1", "0"]]
    else:
        import socket
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        cmd = [[sys.executable, __file__, "--child", str(r), "2", str(port)] for r in range(2)]
    # each child's stderr to a file of its own (a pipe read one child at a time would fill up
    # for the other and stall both ranks inside a collective)
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    files = [os.path.join(out_dir, "dl_probe_rank{}.log".format(r)) for r in range(len(cmd))]
    fhs = [open(f, "w") for f in files]
    procs = [subprocess.Popen(c, env=env, stdout=subprocess.DEVNULL, stderr=fh) for c, fh in zip(cmd, fhs)]
    t0 = time.time()
    while any(p.poll() is None for p in procs):
        time.sleep(5)
        print("... probe running {:.0f} s".format(time.time() - t0), flush=True)
        if time.time() - t0 > 240:
            for p in procs:
                p.kill()
    for fh in fhs:
        fh.close()
    outs = [open(f, errors="replace").read() for f in files]
    rc = [p.returncode for p in procs]
    for r, text in enumerate(outs):
        rows = parse(text)
        print("rank {} (exit {}): {} libraries loaded after the fit started".format(r, rc[r], len(rows)))
        for lib, by, act in rows:
            print("  {:60s} by {:40s} in progress: {}".format(os.path.basename(lib), os.path.basename(by), act or "-"))
    sys.exit(max(abs(x) for x in rc))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
    else:
        main()
