"""Root-cause probe: RCCL's pre-multiplied sum on a bf16 buffer (1-rank RCCL group, one GPU).

Round 4 saw ``dist._make_nccl_premul_sum(2.0)`` return zeros on a bf16 all-reduce.  Hypothesis:
torch hands RCCL the premul scalar as a 4-byte float while declaring the bf16 data type, so RCCL
reads the float's LOW 16 bits as the bf16 factor.  2.0f = 0x40000000 -> low half 0x0000 = bf16 0.0.

The probe all-reduces ones with a premul factor chosen so the two readings differ:

* 2.0                      : float reading 2.0,    low-half reading 0.0
* 0x3F804000 (1.00195...)  : float reading ~1.002, low-half reading bf16 0x4000 = 2.0
* 0x3F803F80 (1.00194...)  : float reading ~1.002, low-half reading bf16 0x3F80 = 1.0

and prints one JSON line per (dtype, factor).  Run under torch.distributed.run with 1 process.
"""
import json
import os
import struct

import torch
import torch.distributed as dist


def f32_from_bits(b: int) -> float:
    return struct.unpack("<f", struct.pack("<I", b))[0]


def main() -> None:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    dev = torch.device("cuda", 0)
    factors = [("2.0", 2.0), ("bits_3F804000", f32_from_bits(0x3F804000)), ("bits_3F803F80", f32_from_bits(0x3F803F80))]
    for dt in (torch.float32, torch.bfloat16):
        for name, f in factors:
            x = torch.ones(4096, dtype=dt, device=dev)
            dist.all_reduce(x, op=dist._make_nccl_premul_sum(f))
            torch.cuda.synchronize()
            vals = sorted(set(float(v) for v in x.float().unique().tolist()))
            print(json.dumps({"dtype": str(dt), "factor": name, "float_value": f, "result_values": vals}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
