"""Helper of tests/test_gpu_rccl.py (test infrastructure, run as its own process): a
torch.distributed process group on the RCCL backend ("nccl") at world size 1 on the box's
GPU, through which the multi-GPU code path runs end to end: dist.solve_sharded (its status
reduction on device tensors under nccl), lvg_solve_layers_device + dist.reduce_status_device
(the bench step's all-reduce) and an all_gather of device populations (solve_sharded's gather
step at world > 1). Writes the results to the .npz named by argv[1]; the parent compares
them with the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out):
    import torch
    import torch.distributed as td
    from radiative_transfer_amd import abi, dist, synth
    from radiative_transfer_amd.native import LvgSolver

    torch.cuda.set_device(0)
    td.init_process_group(backend="nccl")
    assert td.get_backend() == "nccl" and td.get_world_size() == 1
    name, nl = sys.argv[2], int(sys.argv[3])
    P, L, o = synth.make_problem(name, nb_lay=nl)
    opts = abi.default_opts(**o)
    N = P.mol.nb_lev
    s = LvgSolver(P, device=0)
    # host entry through the sharding helper (status reduction on a cuda tensor: RCCL)
    pops, status, totals = dist.solve_sharded(L, lambda Ls: s.solve_layers(Ls, opts), N, gather=True)
    # device entry + the bench step's device all-reduce
    dev = torch.device("cuda", 0)
    soa = torch.from_numpy(L.soa()).to(dev)
    pd = torch.zeros((nl, N), dtype=torch.float64, device=dev)
    sd = torch.zeros((nl, abi.STATUS_DTYPE.itemsize // 8), dtype=torch.float64, device=dev)
    s.solve_layers_device(nl, soa.data_ptr(), pd.data_ptr(), sd.data_ptr(), opts,
                          stream_ptr=torch.cuda.current_stream().cuda_stream)
    tot_d = dist.reduce_status_device(sd)
    gathered = [torch.zeros_like(pd) for _ in range(td.get_world_size())]
    td.all_gather(gathered, pd)
    torch.cuda.synchronize()
    np.savez(out, pops=pops, status=np.frombuffer(status.tobytes(), dtype=np.uint8),
             totals=np.array(totals, dtype=np.float64), tot_d=tot_d.cpu().numpy(), pops_d=gathered[0].cpu().numpy(),
             status_d=np.frombuffer(dist.status_numpy(sd).tobytes(), dtype=np.uint8))
    s.close()
    td.destroy_process_group()
    print("rccl world-1 ok", flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
