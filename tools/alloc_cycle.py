"""hipMalloc/hipFree cycles of one large block (PyTorch's caching allocator
off: PYTORCH_NO_HIP_MEMORY_CACHING=1): the time of each allocation, of a
first touch of the whole block, and of the free.
usage: PYTORCH_NO_HIP_MEMORY_CACHING=1 python tools/alloc_cycle.py [GiB] [reps]"""
import json
import sys
import time

import torch


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 42.0
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    n = int(gib * 2**30)
    torch.cuda.init()
    for k in range(reps):
        t0 = time.perf_counter()
        x = torch.empty(n, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        x[:: 1 << 21].fill_(1)  # one byte per 2 MiB page
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        del x
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        print(json.dumps({"cycle": k, "alloc_ms": round((t1 - t0) * 1e3, 1), "touch_ms": round((t2 - t1) * 1e3, 1),
                          "free_ms": round((t3 - t2) * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
