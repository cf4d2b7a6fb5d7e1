"""Which Python call sites issue device-to-device memcpys (rocclr copyBuffer blits) in one eager
c3 training step: torch.profiler with stacks, the CPU ops whose device work is a memcpy.

    python scripts/find_copies.py
Reference point only: nothing here is on the product path."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402
from jmt import functional as JF  # noqa: E402
from jmt.optim import FusedSGD  # noqa: E402
from losses.loss import CCCLoss  # noqa: E402
from models.two_transformers import Two_transformers  # noqa: E402
from models.fc_layer import FcLayer  # noqa: E402


def main():
    dev = "cuda"
    B, T, Da, Dv, E = 64, 300, 1024, 2048, 512
    torch.manual_seed(0)
    model = Two_transformers(0.0, 0.0, 1, 1, "TRANSFORMER", "FC", Dv).to(dev)
    fc = FcLayer(Da, E).to(dev)
    audio, video, lv, la = bench.synthetic_batch(B, T, Da, Dv, 0, dev)
    crit = CCCLoss(1)
    one = torch.ones((), dtype=torch.float32, device=dev)
    flat = lambda o: o.view(-1, o.shape[0] * o.shape[1])
    opt = FusedSGD(list(model.parameters()) + list(fc.parameters()), lr=1e-3, momentum=0.9,
                   nesterov=True, shadow_dtype=torch.bfloat16, fuse_zero_grad=True)

    def step():
        opt.zero_grad()
        with JF.compute_mode(torch.bfloat16):
            vo, ao = model(fc(audio), video)
            l1 = crit(flat(vo), lv)
            loss = crit.forward_add(flat(ao), la, l1)
            loss.backward(one)
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    n = 0
    for e in prof.events():
        ks = [k for k in getattr(e, "kernels", []) if "opy" in k.name or "emcpy" in k.name]
        if not ks:
            continue
        n += 1
        stack = [s for s in (e.stack or []) if "site-packages" not in s][:8]
        print(f"{e.name} shapes {e.input_shapes} device {[(k.name, k.duration) for k in ks]}")
        for s in stack:
            print("    ", s)
    mem = [e for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA and
           ("emcpy" in e.name or "opyBuffer" in e.name)]
    print(f"{n} CPU ops with copy kernels; device memcpy events: "
          f"{[(e.name, round(e.device_time_total, 1)) for e in mem]}")


if __name__ == "__main__":
    main()
