"""Device time of one fp32 delta mix (``ModelMixer.average_delta``, the bench's N > 1 default wire
for fp32 state) on the headline model: fused HIP passes (csrc/kernels/mix.hip hm_mix_delta3)
against the torch formulation, through a one-rank nccl group on one GPU (the collectives are
RCCL's own calls; at N = 1 they move no bytes over xGMI, so this isolates the pack / merge
passes the mix adds on the device).  Also the overlapped delta-sum merge.

    python benchmarks/mix_delta_probe.py [--bits 20] [--reps 10]
"""
import argparse
import json
import os
import socket
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.parallel import mix as M  # noqa: E402
from hivemall_amd.parallel.dist import DistContext  # noqa: E402


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bits", type=int, default=20)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                            device_id=dev)
    ctx = DistContext(0, 1, 0, dev, "nccl")
    tr = FFMTrainer(f"-classification -factors 4 -num_fields 39 -feature_hashing {a.bits} -seed 3", device=dev)
    tr.init_state(1 << a.bits, 39)
    st = tr.state
    tensors = [st["V"], st["wz"], st["wn"], st["w"], st["bias"]]
    payload = sum(t.numel() * t.element_size() for t in tensors)
    out = {"bits": a.bits, "payload_MB": round(payload / 2**20, 1)}
    for fused in (False, True):
        M._FUSED_DELTA = fused
        m = M.ModelMixer(ctx, min_world=1)
        m.average_delta(tensors)                    # seeds the consensus (a full-precision mean)
        for _ in range(2):
            m.average_delta(tensors)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            m.average_delta(tensors)
        e1.record()
        torch.cuda.synchronize()
        out[f"average_delta_ms_{'fused' if fused else 'torch'}"] = round(e0.elapsed_time(e1) / a.reps, 3)
        ov = M.OverlappedMixer(m, mode="sum")
        ov.start(tensors)
        ov.start(tensors)
        ov.finish()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.reps):
            ov.start(tensors)
        ov.finish()
        e1.record()
        torch.cuda.synchronize()
        out[f"overlapped_sum_mix_ms_{'fused' if fused else 'torch'}"] = round(e0.elapsed_time(e1) / a.reps, 3)
        m.release()
        del m, ov
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
