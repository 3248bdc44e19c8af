"""Bitwise A/B of a CFM_* switch on the training step's gradients: python tools/lnpack_eq.py"""
import os, subprocess, sys
# run the cfg-3 shaped 3-layer training step twice (CFM_LN_PACK=1 / 0) in subprocesses and compare
outs = []
for v in ("1", "0"):
    env = dict(os.environ, CFM_LN_PACK=v)
    f = f"/tmp/lnpack_{v}.pt"
    r = subprocess.run([sys.executable, "tools/lnpack_run.py", f], env=env, capture_output=True, text=True, timeout=300)
    print(v, r.stdout.strip(), r.stderr[-500:] if r.returncode else "")
    if r.returncode:
        sys.exit(1)
    outs.append(f)
import torch
a, b = torch.load(outs[0]), torch.load(outs[1])
bad = [k for k in a if not torch.equal(a[k], b[k])]
print("params", len(a), "differ", len(bad), bad[:5])
sys.exit(1 if bad else 0)
