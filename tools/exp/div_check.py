"""How does ATen on the GPU compute `x / 255.0` (scalar divisor)? Compared bit for bit with the true quotient (CPU
ATen and the native kernel) and with x * fl(1/255)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "torch-optical-flow_amd")]
import torch  # noqa: E402

from optical_flow import _native as N  # noqa: E402

g = torch.Generator().manual_seed(0)
x = torch.cat([torch.arange(256, dtype=torch.float32), torch.rand(1 << 20, generator=g) * 255])
x = x[: (x.numel() // 4) * 4]
dev = torch.device("cuda", 0)
xg = x.to(dev)
gpu_div = (xg / 255.0).cpu()
cpu_div = x / 255.0
recip = x * torch.tensor(1.0 / 255.0, dtype=torch.float32)
y_native, _ = N.normalize_images(xg, xg)
y_aten_gpu = (2 * (xg / 255.0) - 1.0).cpu()
y_cpu = 2 * (x / 255.0) - 1.0
out = {
    "gpu_div_vs_cpu_div_mismatch": int((gpu_div != cpu_div).sum()),
    "gpu_div_vs_recip_mismatch": int((gpu_div != recip).sum()),
    "native_vs_cpu_reference_mismatch": int((y_native.cpu() != y_cpu).sum()),
    "aten_gpu_vs_cpu_reference_mismatch": int((y_aten_gpu != y_cpu).sum()),
    "n": x.numel(),
}
print(json.dumps(out))
