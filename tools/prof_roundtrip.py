"""dev: 16K encode + decode round trip for rocprofv3 --kernel-trace --stats."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hiccup_amd import pipeline
n = int(os.environ.get("RT_N", "16384"))
g = torch.Generator(device="cuda"); g.manual_seed(5)
xs = [torch.randint(0, 256, (n, n, 3), dtype=torch.uint8, device="cuda", generator=g) for _ in range(2)]
enc, dec = pipeline.Encoder(n, n), pipeline.Decoder(n, n)
for i in range(6):
    enc.encode(xs[i % 2])
    counts = enc.counts.cpu().tolist()
    dec.decode(enc.sym_len, enc.sym_val, counts, enc.dc)
torch.cuda.synchronize()
print("done", counts)
