"""Write the tie_probe matrices as jv_clock input files (int32 nr, nc; f64 row-major)."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tie_probe import crowd  # noqa: E402

out = Path(sys.argv[1])
out.mkdir(parents=True, exist_ok=True)
for name, c in [("eq512", np.full((512, 512), 0.5)), ("crowd", crowd()), ("crowd2", crowd(2, 128, 64))]:
    with open(out / f"{name}.bin", "wb") as f:
        np.array(c.shape, np.int32).tofile(f)
        c.astype(np.float64).tofile(f)
