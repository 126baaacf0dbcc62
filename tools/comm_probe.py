"""Multi-process rehearsal of the library's RCCL communicator (mmb_comm_init with a unique id,
one engine per process).  Launch with
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/comm_probe.py
On a one-GPU box both ranks share device 0, which RCCL may refuse; the script reports that.
Rank 0 prints the PSRF from mmb_gr_allreduce next to the host gelmandiag of all chains."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = rank % max(torch.cuda.device_count(), 1)
    import _mamba_path
    mb = _mamba_path.load()
    K = 256
    m = mb.rats()
    m.setinputs(mb.model.RATS_DATA)
    m.setsamplers(mb.model.rats_scheme_gibbs_amm())
    init = mb.model.rats_init_ls(K * world, seed=3)
    eng = mb.Engine(m, device=dev)
    eng.init_chains(init[rank * K:(rank + 1) * K], chain_offset=rank * K, seed=4)
    eng.run(200, burnin=40, thin=2, keep_device=True)
    obj = [mb.Comm.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    try:
        comm = mb.Comm([eng], nranks=world, rank0=rank, uid=obj[0])
    except RuntimeError as ex:
        print(f"rank {rank}: communicator refused: {ex}", flush=True)
        dist.destroy_process_group()
        return
    ps, mp = mb.gelmandiag_rccl(comm, mpsrf=True)
    comm.close()
    if rank == 0:
        e1 = mb.Engine(m, device=dev)
        e1.init_chains(init, seed=4)
        d = e1.run(200, burnin=40, thin=2, keep_device=True)
        ps_h, mp_h = mb.gelmandiag(d, mpsrf=True)
        print("rccl psrf", ps[:, 0].tolist(), "host psrf", ps_h[:, 0].tolist(),
              "max rel diff", float(np.abs(ps / ps_h - 1).max()), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
