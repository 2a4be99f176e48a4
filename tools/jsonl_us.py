#!/usr/bin/env python3
"""Dev tool: one compact line `config=us ...` from a bench_configs JSONL file."""
import json
import sys

print(" ".join(f"{d['config']}={d['us']}" for d in map(json.loads, open(sys.argv[1]))))
