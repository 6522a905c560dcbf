"""PMC calibration probe: a 1 GiB device-to-device copy (well past the 256 MiB Infinity Cache), so FETCH_SIZE /
WRITE_SIZE of its dispatch can be compared with the known 1 GiB read + 1 GiB write."""
import torch

x = torch.ones(1 << 29, dtype=torch.bfloat16, device="cuda")
y = torch.empty_like(x)
for _ in range(3):
    y.copy_(x)
torch.cuda.synchronize()
print("copied", x.numel() * 2, "bytes x3")
