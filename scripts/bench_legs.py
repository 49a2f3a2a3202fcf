"""Print the c3 value and the c2 / c5 legs of a bench.py JSON line read from stdin (A/B scripts)."""
import json
import sys

d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print(d["value"], d.get("c2_latency_s"), d.get("c5_images_per_s"), flush=True)
