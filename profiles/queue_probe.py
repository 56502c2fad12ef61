"""Which HSA queue does each kind of stream land on?  (run under rocprofv3 --kernel-trace)

One small fill kernel per stream kind, tagged by its element count, so the kernel trace's
Queue_Id column shows the queue of each: torch's default stream, a new torch stream, a
high-priority torch stream, a stream created with a full CU mask (hipExtStreamCreateWithCUMask),
and RCCL's stream (an all_reduce; world 1, under torch.distributed env:// variables).
"""
import ctypes as C
import os
import sys

import torch
import torch.distributed as dist

torch.cuda.set_device(0)
dev = torch.device("cuda:0")
hip = C.CDLL("libamdhip64.so")


def cu_mask_stream():
    s = C.c_void_p()
    mask = (C.c_uint32 * 8)(*([0xFFFFFFFF] * 8))  # every CU
    rc = hip.hipExtStreamCreateWithCUMask(C.byref(s), 8, mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


def tag(stream, n, label):
    with torch.cuda.stream(stream):
        torch.empty(n, device=dev).fill_(1.0)
    print(f"{label}: fill of {n} elements", file=sys.stderr)


early = cu_mask_stream()  # before torch's stream pools exist
dist.init_process_group("nccl", device_id=dev)
tag(torch.cuda.default_stream(dev), 1001, "default stream")
tag(torch.cuda.Stream(dev), 1002, "new torch stream")
tag(torch.cuda.Stream(dev, priority=-1), 1003, "high-priority torch stream")
tag(early, 1004, "CU-mask stream created before init_process_group")
tag(cu_mask_stream(), 1005, "CU-mask stream created after")
x = torch.ones(1 << 20, device=dev)
dist.all_reduce(x)
dist.all_reduce(x, async_op=True).wait()
torch.cuda.synchronize()
print("all_reduce done", file=sys.stderr)
dist.destroy_process_group()
