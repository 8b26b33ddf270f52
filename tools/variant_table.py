"""Summarise bench.py logs of library variants (tooling): for each gpurun_out/<name>.log given,
the per-k forward / backward times of its last JSON line.

  python tools/variant_table.py gpurun_out/v_base.log gpurun_out/v_x.log ...
"""
import json
import sys


def main():
    for path in sys.argv[1:]:
        try:
            lines = [l for l in open(path) if l.startswith("{")]
        except OSError as exc:
            print(path, "missing:", exc)
            continue
        if not lines:
            print(path, "no result")
            continue
        d = json.loads(lines[-1])
        sweep = d.get("k_sweep") or {str(d["config"]["dim_k"]): d}
        cells = " ".join(f"k{k}:{v['fwd_ms']:.4f}/{v['bwd_ms']:.4f}" for k, v in sweep.items())
        print(f"{path}: {cells}  lib {d['roofline'].get('lib_sha256', '')[:12]}")


if __name__ == "__main__":
    main()
