"""dev: the bench's 16K round trip extra alone (for rocprofv3 --kernel-trace)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

print(json.dumps(bench.extra_16k_roundtrip(steps=3)))
