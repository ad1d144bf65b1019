"""Can RCCL run a world of two ranks on a one-GPU box?  Two processes, both on cuda:0:

1. ``torch.distributed`` "nccl" (RCCL) init + one fp64 all-reduce of the shared block's size;
2. the library's own communicator (``engine.RcclComm``, pert_comm_init) + one all-reduce.

NCCL refuses two ranks on one device ("Duplicate GPU detected"); this records what this RCCL
does.  Each rank prints one line; the parent prints a JSON summary.  Every step runs under a
deadline in the children (faulthandler dump at 40 s, hard exit at 50 s).

usage: python tools/rccl_two_ranks.py
"""
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _worker(rank, world, port, out):
    import faulthandler
    import threading
    faulthandler.dump_traceback_later(40, exit=False)
    threading.Timer(50, lambda: os._exit(3)).start()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    res = {"rank": rank}
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    try:
        dist.init_process_group("nccl", device_id=dev)
        t = torch.full((5452,), float(rank + 1), dtype=torch.float64, device=dev)
        t0 = time.perf_counter()
        dist.all_reduce(t)
        torch.cuda.synchronize()
        res["torch_allreduce"] = {"ok": bool(torch.all(t == 3.0).item()), "s": time.perf_counter() - t0}
    except Exception as e:                                       # noqa: BLE001 (record what RCCL says)
        res["torch_allreduce"] = {"error": repr(e)[:400]}
    try:
        from scdna_replication_tools_amd.engine import RcclComm
        if not dist.is_initialized():
            dist.init_process_group("gloo")
        comm = RcclComm()
        t = torch.full((5452,), float(rank + 1), dtype=torch.float64, device=dev)
        comm.allreduce(t)
        torch.cuda.synchronize()
        res["pert_comm"] = {"ok": bool(torch.all(t == 3.0).item())}
        comm.close()
    except Exception as e:                                       # noqa: BLE001
        res["pert_comm"] = {"error": repr(e)[:400]}
    with open(out.format(rank), "w") as fh:
        json.dump(res, fh)
    try:
        dist.destroy_process_group()
    except Exception:                                            # noqa: BLE001
        pass
    os._exit(0)


def main():
    import torch.multiprocessing as mp
    out = os.path.join(ROOT, "gpurun_out", "rccl_two_ranks_rank{}.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.spawn(_worker, args=(2, port, out), nprocs=2, join=False)
    t0 = time.time()
    while True:
        try:
            if ctx.join(timeout=5):
                break
        except Exception as e:                                   # noqa: BLE001 (a rank exited non-zero)
            print("rank exit:", repr(e)[:300], flush=True)
            break
        if time.time() - t0 > 70:
            for p in ctx.processes:
                if p.is_alive():
                    p.kill()
            break
    ranks = []
    for r in range(2):
        try:
            ranks.append(json.load(open(out.format(r))))
        except OSError:
            ranks.append({"rank": r, "error": "no result (killed or crashed)"})
    print(json.dumps({"what": "RCCL world 2 on one GPU", "ranks": ranks}), flush=True)


if __name__ == "__main__":
    main()
