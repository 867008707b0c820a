"""One rank of a process-per-GPU job for tests/test_distributed.py.

    python tests/dist_worker.py --rank R --world N --port P --out DIR --case CASE

The ranks meet over torch.distributed (gloo, 127.0.0.1) and hand the product a
radler.distributed.HostCommunicator whose collectives are gloo's: several
ranks can then share one GPU (RCCL refuses that), which is how the
distributed ParallelDeconvolution is tested on a one-GPU machine. Results go
to DIR/rank{R}.npz.
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

PIXEL_SCALE = 1.0 / 3600.0 * np.pi / 180.0


def host_communicator(rd, rank, world):
    import torch
    import torch.distributed as dist

    def broadcast(arr, root):
        dist.broadcast(torch.from_numpy(arr), src=root)

    def allreduce_max(v):
        t = torch.tensor([v], dtype=torch.float32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    return rd.distributed.HostCommunicator(world, rank, broadcast, allreduce_max)


def tiled_settings(rd, kind, w, thr, max_iter, mgain, gw, gh):
    s = rd.Settings()
    s.algorithm_type = (rd.AlgorithmType.multiscale if kind == 1
                        else rd.AlgorithmType.generic_clean)
    s.trimmed_image_width = s.trimmed_image_height = w
    s.pixel_scale.x = s.pixel_scale.y = PIXEL_SCALE
    s.minor_iteration_count = max_iter
    s.absolute_threshold = thr
    s.border_ratio = 0.0
    s.major_loop_gain = mgain
    s.parallel.grid_width, s.parallel.grid_height = gw, gh
    if kind == 1:
        s.multiscale.max_scales = 4
    return s


def tiled_problem(w, gw, channels):
    """(psf, dirty) of the distributed tiled tests: one field, or `channels`
    joined channels of one sky (100 MHz + 10 MHz steps, spectral index -0.7,
    a PSF per channel; tests/config_problems.joined_channels)."""
    if channels == 1:
        from synthetic import problem
        return problem(w, w, 40, 4, seed=w + gw)
    from config_problems import joined_channels
    freqs = [100e6 + 10e6 * i for i in range(channels)]
    return joined_channels(w, 40, 4, seed=w + gw, frequencies=freqs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--case", default="host")
    ap.add_argument("--kind", type=int, default=1)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--grid", type=int, nargs=2, default=(2, 2))
    ap.add_argument("--majors", type=int, default=2)
    ap.add_argument("--channels", type=int, default=1,
                    help="joined channels (tests/config_problems.joined_channels)")
    args = ap.parse_args()

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(args.port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=args.rank, world_size=args.world)
    from radler_import import radler as rd
    comm = host_communicator(rd, args.rank, args.world)
    out = {}
    if args.case == "host":
        # the job-side plumbing: broadcast of a host buffer and the max
        a = np.zeros(1 << 16, np.uint8)
        if args.rank == args.world - 1:
            a[:] = (np.arange(a.size) * 7 + 3) % 251
        comm.broadcast_host(a, args.world - 1)
        out["bcast"] = a
        out["max"] = np.float32(comm.allreduce_max(float(args.rank) * 1.5 - 7.0))
        out["owners"] = np.array([rd.distributed.subimage_owner(i, args.world)
                                  for i in range(10)])
    elif args.case == "channels":
        # ONE joined image set (grid 1 x 1) whose per-channel work the ranks
        # share (MultiScaleAlgorithm::SetChannelShard)
        w = args.size
        psf, dirty = tiled_problem(w, 1, args.channels)
        thr, max_iter = 4e-3, 1500
        mgain = 0.9 if args.majors == 1 else 0.5
        s = tiled_settings(rd, 1, w, thr, max_iter, mgain, 1, 1)
        run = rd.gpu.DeviceRun(s, psf, dirty, [1.0] * args.channels, 2.0 * PIXEL_SCALE)
        run.set_communicator(comm)
        for major in range(args.majors):
            r = run.execute()
            out[f"residual{major}"] = run.residual()
            out[f"model{major}"] = run.model()
            out[f"iterations{major}"] = np.int64(r["iterations"])
            out[f"another{major}"] = np.int64(r["another_iteration_required"])
            out[f"trace{major}"] = run.trace(0)
        run.sync()
        del run
    else:
        w = args.size
        gw, gh = args.grid
        psf, dirty = tiled_problem(w, gw, args.channels)
        thr, max_iter = 4e-3, 1500
        mgain = 0.9 if args.majors == 1 else 0.5
        s = tiled_settings(rd, args.kind, w, thr, max_iter, mgain, gw, gh)
        run = rd.gpu.DeviceRun(s, psf, dirty, [1.0] * args.channels if args.channels > 1 else [],
                               2.0 * PIXEL_SCALE if args.kind == 1 else 0.0)
        run.set_communicator(comm)
        for major in range(args.majors):
            r = run.execute()
            out[f"residual{major}"] = run.residual()
            out[f"model{major}"] = run.model()
            out[f"iterations{major}"] = np.int64(r["iterations"])
            out[f"another{major}"] = np.int64(r["another_iteration_required"])
            owners = run.clean_owners()  # cost-ordered (LPT) cleaning-pass owners
            out[f"owners{major}"] = np.array(owners, np.int64)
            for i in range(gw * gh):
                if owners[i] == args.rank:
                    out[f"trace{major}_{i}"] = run.trace(i)
        run.sync()
        del run
    np.savez(os.path.join(args.out, f"rank{args.rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
