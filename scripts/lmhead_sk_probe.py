"""Which hipBLASLt kernels do the LM head's GEMMs pick for N = 12388 tokens, chunk 4096
(3 full chunks + a 100-row ragged chunk)? Run SEQUENTIALLY on one stream (safe) under
``rocprofv3 --kernel-trace --stats`` to see whether the torch GEMMs that the removed
side-stream-dW layout ran concurrently are stream-K (``_SK<n>``) kernels."""
import torch

from ray_amd.ops import lt

dev = torch.device("cuda", 0)
C, Vp = 768, 50304
w = torch.randn(Vp, C, device=dev).bfloat16()
for rows in (4096, 100):
    h = torch.randn(rows, C, device=dev).bfloat16()
    lg = h @ w.t()                                   # logits  [rows, Vp]
    dh = lg @ w                                      # dh      [rows, C]
    dw = torch.zeros(Vp, C, device=dev)
    torch.addmm(dw, lg.t(), h, out_dtype=torch.float32, out=dw)  # old side-stream dW
    torch.cuda.synchronize()
    name = lt.wgrad_choice_name(rows, Vp, C, 1)
    print(f"rows={rows}: ops/lt dW kernel = {name} streamk={lt.is_streamk(name)}", flush=True)
