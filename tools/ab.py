"""A/B driver for GPU measurements: runs benchmark commands under several variants,
interleaved, and tabulates the JSON lines they print.

A variant is ``label`` or ``label:ENV=VALUE[,ENV=VALUE...]``; ``LIGHTGBM_AMD_LIB=path`` selects a
variant library (tools/build_variant.sh).  Each --bench is a command run from the repository
root (``python`` is prepended when it starts with a .py file); every (bench, variant) pair is
repeated --reps times in the order bench x rep x variant, so the variants of one rep run back
to back.  Each run has its own time limit and a failing run ends the driver (nonzero exit), as
the GPU box's rules ask.

  python tools/ab.py --out gpurun_out/k --reps 2 \\
      --bench "bench.py --steps 100 --warmup 5 --test-rows 0" \\
      --bench "bench.py --rows 1250000 --steps 100 --warmup 5 --test-rows 0" \\
      --variant k8 --variant k6:LGBM_AMD_ROUND_K=6

Prints one line per run and a markdown table of the mean of each field (--fields) per bench and
variant; writes the logs and summary.md under --out.
"""
import argparse
import json
import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse_variant(text):
    label, _, env = text.partition(":")
    out = {}
    for kv in filter(None, env.split(",")):
        k, _, v = kv.partition("=")
        out[k] = v
    return label, out


def last_json(text):
    for line in reversed(text.splitlines()):
        line = line.strip()
        if line.startswith("{") and line.endswith("}"):
            try:
                return json.loads(line)
            except ValueError:
                continue
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--bench", action="append", required=True)
    ap.add_argument("--variant", action="append", default=[])
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--timeout", type=int, default=300, help="seconds per run")
    ap.add_argument("--fields", default="ms_per_step,rounds_per_tree")
    args = ap.parse_args()
    variants = [parse_variant(v) for v in (args.variant or ["base"])]
    fields = [f for f in args.fields.split(",") if f]
    os.makedirs(args.out, exist_ok=True)
    results = {}
    for bi, bench in enumerate(args.bench):
        cmd = shlex.split(bench)
        if cmd[0].endswith(".py"):
            cmd = [sys.executable, "-u"] + cmd
        for rep in range(args.reps):
            for label, env in variants:
                log = os.path.join(args.out, "b%d_%s_r%d.log" % (bi, label, rep))
                t0 = time.time()
                with open(log, "w") as f:
                    try:
                        rc = subprocess.run(["timeout", "-k", "10", str(args.timeout)] + cmd, cwd=ROOT,
                                            env=dict(os.environ, **env), stdout=f, stderr=subprocess.STDOUT).returncode
                    except KeyboardInterrupt:
                        raise
                rec = last_json(open(log).read())
                if rc != 0 or rec is None:
                    print("[%s] bench %d rep %d failed (rc %d): see %s" % (label, bi, rep, rc, log), flush=True)
                    sys.exit(1)
                vals = {k: rec.get(k) for k in fields}
                results.setdefault((bi, label), []).append(vals)
                print("[%s] bench %d rep %d %.0fs %s" % (label, bi, rep, time.time() - t0,
                                                         " ".join("%s=%s" % kv for kv in vals.items())), flush=True)
    lines = ["| bench | variant | " + " | ".join(fields) + " |", "|---|---|" + "---|" * len(fields)]
    for (bi, label), runs in results.items():
        cells = []
        for k in fields:
            xs = [r[k] for r in runs if isinstance(r.get(k), (int, float))]
            cells.append("%.4g" % (sum(xs) / len(xs)) if xs else "-")
        lines.append("| `%s` | %s | %s |" % (args.bench[bi], label, " | ".join(cells)))
    summary = "\n".join(lines)
    print(summary)
    with open(os.path.join(args.out, "summary.md"), "w") as f:
        f.write(summary + "\n")


if __name__ == "__main__":
    main()
