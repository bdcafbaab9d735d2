"""Training logs in the reference's formats.

The reference logs through stable-baselines3's `configure(path, ["stdout",
"csv"])` (train.py:216-218): a `progress.csv` whose columns appear in the order
keys are first recorded (new keys extend the header and pad earlier rows with
empty cells, SB3 CSVOutputFormat), plus a stdout table per dump.  The archived
runs' progress.csv files (outputs/experiments/archived_models/*/progress.csv)
have exactly these columns: time/*, rollout/ep_rew_mean, rollout/ep_len_mean,
train/* and eval/*.  This logger writes the same file so the reference's
plotting scripts (ballbot_rl/visualization/plot_training.py) read it unchanged.
"""
from __future__ import annotations

import sys
from pathlib import Path
from typing import Any, Dict, List, Optional


class CSVLogger:
    """SB3-compatible key/value logger: record() values, dump() one row."""

    def __init__(self, folder: Optional[str] = None, stdout: bool = True, csv_name: str = "progress.csv"):
        self.values: Dict[str, Any] = {}
        self.keys: List[str] = []
        self.rows: List[Dict[str, Any]] = []
        self.stdout = stdout
        self.path = None
        if folder:
            Path(folder).mkdir(parents=True, exist_ok=True)
            self.path = Path(folder) / csv_name

    def record(self, key: str, value: Any) -> None:
        self.values[key] = value

    def record_mean(self, key: str, values) -> None:
        vals = list(values)
        if vals:
            self.values[key] = float(sum(vals) / len(vals))

    def dump(self, step: int = 0) -> None:
        if not self.values:
            return
        new = [k for k in self.values if k not in self.keys]
        self.keys.extend(new)
        self.rows.append(dict(self.values))
        if self.path is not None:
            self._write(rewrite=bool(new) or len(self.rows) == 1)
        if self.stdout:
            self._print()
        self.values = {}

    def _fmt(self, v: Any) -> str:
        if v is None:
            return ""
        if isinstance(v, str):
            return '"' + v.replace('"', '""') + '"'
        return str(v)

    def _write(self, rewrite: bool) -> None:
        if rewrite:
            with self.path.open("w") as f:
                f.write(",".join(self.keys) + "\n")
                for r in self.rows:
                    f.write(",".join(self._fmt(r.get(k)) for k in self.keys) + "\n")
        else:
            with self.path.open("a") as f:
                f.write(",".join(self._fmt(self.rows[-1].get(k)) for k in self.keys) + "\n")

    def _print(self) -> None:
        r = self.rows[-1]
        w = max(len(k) for k in r) + 2
        lines = ["-" * (w + 16)]
        for k in sorted(r):
            v = r[k]
            s = f"{v:.4g}" if isinstance(v, float) else str(v)
            lines.append(f"| {k:<{w}}| {s:<12}|")
        lines.append("-" * (w + 16))
        print("\n".join(lines), file=sys.stdout, flush=True)


def read_progress(path: str) -> Dict[str, List[Optional[float]]]:
    """progress.csv -> column -> values (None for empty cells); reads the reference's files too."""
    import csv

    with open(path) as f:
        rows = list(csv.DictReader(f))
    cols: Dict[str, List[Optional[float]]] = {}
    for r in rows:
        for k, v in r.items():
            try:
                cols.setdefault(k, []).append(float(v) if v not in ("", None) else None)
            except ValueError:
                cols.setdefault(k, []).append(None)
    return cols
