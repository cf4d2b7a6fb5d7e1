"""Narrow the multi-stream capture crash on the real model: case fwd | fwdbwd | step."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd")]
import torch
from jmt import functional as JF
from models.two_transformers import Two_transformers
from models.fc_layer import FcLayer
from losses.loss import CCCLoss

case = sys.argv[1]
dev = torch.device("cuda")
B, T = 4, 37
m = Two_transformers(0.0, 0.0, 1, 1, "TRANSFORMER", "FC", 2048).to(dev)
fc = FcLayer(1024, 512).to(dev)
audio = torch.randn(B, T, 1024, device=dev)
video = torch.randn(B, T, 2048, device=dev)
lv = torch.rand(1, B * T, device=dev)
crit = CCCLoss(1)


def body():
    with JF.compute_mode(torch.bfloat16):
        if case == "fwd":
            with torch.no_grad():
                vo, ao = m(fc(audio), video)
            return vo
        if case == "enc":
            x = torch.randn(T, B, 512, device=dev)
            with torch.no_grad():
                return m.mm_transformer.visual_encoder(x)
        vo, ao = m(fc(audio), video)
        loss = crit(vo.reshape(1, -1), lv) + crit(ao.reshape(1, -1), lv)
        loss.backward()
        return loss


side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(2):
        body()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
print("warm ok", flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, capture_error_mode=os.environ.get("CAPMODE", "global")):
    out = body()
print("captured", flush=True)
torch.cuda.synchronize()
g.replay()
torch.cuda.synchronize()
print(case, "OK", float(out.float().sum()), flush=True)
