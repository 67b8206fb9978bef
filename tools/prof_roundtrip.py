"""dev: the 16K encode + decode round trip for rocprofv3 --kernel-trace --stats, on
the product path (the slot-layout encode, the decode from its record index with the
counts on the device).  RT_N: the image side (default 16384)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hiccup_amd import pipeline  # noqa: E402

n = int(os.environ.get("RT_N", "16384"))
g = torch.Generator(device="cuda")
g.manual_seed(5)
xs = [torch.randint(0, 256, (n, n, 3), dtype=torch.uint8, device="cuda", generator=g) for _ in range(2)]
enc, dec = pipeline.Encoder(n, n, index=True), pipeline.Decoder(n, n)
for i in range(6):
    enc.encode(xs[i % 2])
    dec.decode(enc.sym_len, enc.sym_val, enc.counts, enc.dc, index=enc.index)
torch.cuda.synchronize()
dec.check_status()
print("done", enc.slots, enc.counts.cpu().tolist())
