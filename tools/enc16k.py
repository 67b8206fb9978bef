"""dev: 16K encodes on one stream (for a kernel trace of the encode half of the
round trip); HICCUP_HIP_LIB selects the library."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hiccup_amd import pipeline  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
g = torch.Generator(device="cuda")
g.manual_seed(5)
x = torch.randint(0, 256, (n, n, 3), dtype=torch.uint8, device="cuda", generator=g)
enc = pipeline.Encoder(n, n, index=True)
for _ in range(8):
    enc.encode(x)
torch.cuda.synchronize()
print("ok", [int(c) for c in enc.counts.cpu()])
