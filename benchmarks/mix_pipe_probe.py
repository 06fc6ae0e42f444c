"""Device time of one mix of the headline FFM model, monolithic vs bucketed + pipelined
(``ModelMixer._pipelined``), through a one-rank nccl group on one GPU: RCCL's
own all_to_all / all_gather calls (device copies at N = 1, no xGMI bytes) on RCCL's stream next to
the fused pack / shard-mean / merge passes on the compute stream.  ms per mix = events around
``reps`` back-to-back mixes on the compute stream, i.e. the device time a mix holds the
training stream.

    python benchmarks/mix_pipe_probe.py [--bits 20] [--reps 10] [--buckets 0,16,32,64]
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
from hivemall_amd.ops.ffm import linear_mix_tensors  # noqa: E402
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
    ap.add_argument("--buckets", default="0,16,32,64")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                            device_id=dev)
    ctx = DistContext(0, 1, 0, dev, "nccl")
    for state in ("fp32", "bf16"):
        tr = FFMTrainer(f"-classification -factors 4 -num_fields 39 -feature_hashing {a.bits} -seed 3"
                        + (" -bf16_state" if state == "bf16" else ""), device=dev)
        tr.init_state(1 << a.bits, 39)
        st = tr.state
        tensors = [st["V"], *linear_mix_tensors(st), st["bias"]]
        payload = sum(t.numel() * t.element_size() for t in tensors)
        for mb in [float(x) for x in a.buckets.split(",")]:
            m = M.ModelMixer(ctx, min_world=1)
            m.PIPE_BUCKET_MB = mb
            fn = m.average_delta if state == "fp32" else m.average
            for _ in range(3):
                fn(tensors)                       # (average_delta: the first call seeds the consensus)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                fn(tensors)
            e1.record()
            torch.cuda.synchronize()
            grp = [p for k, p in m._plans.items() if k[0] == "delta"] or list(m._plans.values())
            grp = grp[0][0]
            nb = len(grp.buckets(int(mb * (1 << 20)) // grp.send.element_size())) if mb else 1
            print(json.dumps({"state": state, "fn": fn.__name__, "payload_MB": round(payload / 2**20, 1),
                              "wire_MB": round(grp.nbytes / 2**20, 1), "bucket_MB": mb, "buckets": nb,
                              "ms_per_mix": round(e0.elapsed_time(e1) / a.reps, 3)}), flush=True)
            m.release()
            del m
            torch.cuda.empty_cache()
        del tr, st, tensors
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
