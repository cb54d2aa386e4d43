"""Dev aid: bench.py's reference_call_pattern measurement alone (one QP per solve())."""
import importlib.util
import json
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
pkg = bench.import_pkg()
print(json.dumps(bench.call_pattern(pkg, 1003)))
