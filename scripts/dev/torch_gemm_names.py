"""torch.bmm on two of the step's shapes (the ones that ran cleanly) so rocprofv3 can record which
hipBLASLt kernels (macro tile, MFMA, wave layout in the name) the vendor library picks."""
import torch
R = 19200
bf = torch.bfloat16
A = torch.randn(3, R, 512, device="cuda", dtype=bf)
W = torch.randn(3, 512, 512, device="cuda", dtype=bf)
for _ in range(5):
    torch.bmm(A, W.transpose(1, 2))
    torch.bmm(A, W)
torch.cuda.synchronize()
print("ok")
