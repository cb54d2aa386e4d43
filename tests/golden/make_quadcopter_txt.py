"""Write quadcopter_AB.txt (row-major A then B of the compareResults fixture in
quadcopter.json) for the C++ hpipm-cpp interface tests, which have no JSON
parser.  Data only: two lines of whitespace-separated numbers."""
import json
from pathlib import Path

here = Path(__file__).resolve().parent
d = json.loads((here / "quadcopter.json").read_text())
with open(here / "quadcopter_AB.txt", "w") as f:
    for key in ("A", "B"):
        f.write(" ".join(repr(float(v)) for row in d[key] for v in row) + "\n")
