"""Probe: can an RCCL collective be captured in a HIP graph on this image?  One-rank `nccl` group on
cuda:0; variants (argv[2]): "pg" -- torch's dist.all_reduce inside torch.cuda.graph (thread-local
capture mode); "direct" -- ncclAllReduce called through ctypes on torch's own librccl.so with the
process group's communicator (_comm_ptr) on the capturing stream.  Prints one line per variant."""
import ctypes
import faulthandler
import os
import sys

import torch
import torch.distributed as dist


def main():
    faulthandler.enable()
    port, variant = int(sys.argv[1]), sys.argv[2]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1, device_id=dev)
    x = torch.arange(1024, dtype=torch.float32, device=dev)
    y = x * 2
    dist.all_reduce(y)  # eager: creates the communicator
    torch.cuda.synchronize()
    print("eager ok", bool(torch.equal(y, x * 2)), flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    if variant == "pg":
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            y = x * 3
            dist.all_reduce(y)
    else:
        lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"))
        comm = dist.group.WORLD._get_backend(dev)._comm_ptr()
        print("comm", hex(comm), flush=True)
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            y = x * 3
            st = lib.ncclAllReduce(ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                                   ctypes.c_size_t(y.numel()), ctypes.c_int(7), ctypes.c_int(0),
                                   ctypes.c_void_p(comm), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        print("nccl status", st, flush=True)
    print("captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print("replay ok", variant, bool(torch.equal(y, x * 3)), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
