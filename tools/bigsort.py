"""The bench's beyond-cache sort alone (bench.sort_bench_big: 64M uniform pairs) and the
sortTests-input sort, printed as JSON.  python tools/bigsort.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import openglgaussiansplattingrenderer_amd as g  # noqa: E402

ctx = g.Context(0)
print(json.dumps(bench.sort_bench_big(ctx)), flush=True)
