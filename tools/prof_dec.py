"""Profile driver (dev tool): one n x n encode with the tile index, then `reps`
decodes (pipeline.Decoder.decode with index=); argv[3] = 1: keep_blocks (the
indexed decode writes the zig-zag blocks, then hic_dequant_idct_u8), else the
fused hic_rle_decode_idct_u8_indexed.  Prints the median wall time per decode.
usage: python3 tools/prof_dec.py [n=16384] [reps=4] [keep_blocks=0] [planes=0] [chroma_pair=1]
(planes=1: the Y plane and the separate colour kernel, as libraries before
hic_rle_decode_idct_rgb_indexed)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hiccup_amd import pipeline  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
keep = bool(int(sys.argv[3])) if len(sys.argv) > 3 else False
planes = bool(int(sys.argv[4])) if len(sys.argv) > 4 else False
pair = bool(int(sys.argv[5])) if len(sys.argv) > 5 else True  # Decoder chroma_pair
g = torch.Generator(device="cuda")
g.manual_seed(5)
x = torch.randint(0, 256, (n, n, 3), dtype=torch.uint8, device="cuda", generator=g)
enc, dec = pipeline.Encoder(n, n, index=True), pipeline.Decoder(n, n, chroma_pair=pair)
enc.encode(x)
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    t0 = time.perf_counter()
    out = dec.decode(enc.sym_len, enc.sym_val, enc.counts, enc.dc, index=enc.index, keep_blocks=keep, planes=planes)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
dec.check_status()
ts.sort()
print("decode %dx%d keep_blocks=%d planes=%d pair=%d: median %.3f ms, checksum %d, symbols %s" %
      (n, n, keep, planes, pair, ts[len(ts) // 2] * 1e3, int(out[::97, ::89].float().sum().item()), enc.counts.tolist()))
