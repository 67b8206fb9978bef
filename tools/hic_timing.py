"""dev: time codec.jpeg_encode's whole chain at 8K on the GPU -- the encode
(pipeline.Encoder) plus the Huffman back end (Encoder.hic_image: GPU key
histograms, host heapq trees, GPU bit packing) and the container bytes."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hiccup_amd import pipeline  # noqa: E402


def main():
    H, W = 4320, 7680
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    x = torch.randint(0, 256, (H, W, 3), dtype=torch.uint8, device="cuda", generator=g)
    enc = pipeline.Encoder(H, W)
    for i in range(4):
        enc.encode(x)
        t0 = time.perf_counter()
        img = enc.hic_image()
        t1 = time.perf_counter()
        b = img.byte_stream()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        print("hic_image %.1f ms, container byte stream %d bytes (%.1f ms)" % (
            (t1 - t0) * 1e3, sum(len(x) for x in b), (t2 - t1) * 1e3), flush=True)




def profile():
    import cProfile
    import pstats
    H, W = 4320, 7680
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    x = torch.randint(0, 256, (H, W, 3), dtype=torch.uint8, device="cuda", generator=g)
    enc = pipeline.Encoder(H, W)
    enc.encode(x)
    enc.hic_image()
    enc.encode(x)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    img = enc.hic_image()
    img.byte_stream()
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(30)


if __name__ == "__main__":
    profile() if "--profile" in sys.argv else main()
