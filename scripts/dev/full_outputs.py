"""Dev aid: bench.py's unconstr_n20_full_outputs line alone (for a kernel trace)."""
import importlib.util
import json
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
import torch  # noqa: E402

pkg = bench.import_pkg()
print(json.dumps(bench.full_outputs_line(pkg, pkg.capi, torch.device("cuda", 0), 1003)))
