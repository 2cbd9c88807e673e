"""Root-causing round 1's TunableOp NaN (profiles/r01/tunableop/bench_with_tunableop_nan_loss.json).

For every GEMM shape TunableOp tuned in round 1 (profiles/r01/tunableop/results0.csv), replay the
recorded solution (tuning off, the CSV as the selection file) on random bf16 operands of the same
shape, in the three forms conv1x1.py has used: mm, the in-place accumulate addmm_ (C aliases D,
round 1's default) and the out-of-place addmm (this round). Each is compared with the same op
with TunableOp off (the default engine) and with an fp32 reference; one JSON line per case."""
from __future__ import annotations

import csv
import json
import os
import re
import sys

import torch

CSV = sys.argv[1] if len(sys.argv) > 1 else "profiles/r01/tunableop/results0.csv"
dev = torch.device("cuda", 0)


def shapes():
    for row in csv.reader(open(CSV)):
        if not row or row[0] == "Validator":
            continue
        op, sig, sol = row[0], row[1], row[2]
        m = re.match(r"(nn|tn|nt)_(\d+)_(\d+)_(\d+)_ld", sig)
        if not m or "Bias" in op:
            continue
        yield m.group(1), int(m.group(2)), int(m.group(3)), int(m.group(4)), sol


def run_all(tunable: bool):
    torch.cuda.tunable.enable(tunable)
    if tunable:
        torch.cuda.tunable.tuning_enable(False)
        torch.cuda.tunable.set_filename(CSV, insert_device_ordinal=False)
        torch.cuda.tunable.read_file(CSV)
    out = {}
    for lay, m, n, k, sol in shapes():
        g = torch.Generator(device=dev).manual_seed(m * 7 + n * 3 + k)
        # column-major C[m x n] = op(A)[m x k] op(B)[k x n]  <->  row-major D[n x m] = B'[n x k] A'[k x m]
        if lay == "nn":      # dgrad: dx[M, cin] = g2[M, cout] @ wc[cout, cin]; M = n, cin = m, cout = k
            A = torch.randn(n, k, device=dev, generator=g).to(torch.bfloat16)
            B = torch.randn(k, m, device=dev, generator=g).to(torch.bfloat16)
        else:                # tn: fwd y[M, cout] = x2[M, cin] @ wc[cout, cin]^T; M = n, cout = m, cin = k
            A = torch.randn(n, k, device=dev, generator=g).to(torch.bfloat16)
            B = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16).t()
        C = torch.randn(n, m, device=dev, generator=g).to(torch.bfloat16)
        res = {"mm": torch.mm(A, B)}
        if lay == "nn":
            res["addmm_inplace"] = C.clone().addmm_(A, B)
            res["addmm_outofplace"] = torch.addmm(C, A, B)
        ref = A.float() @ B.float()
        out[(lay, m, n, k)] = (sol, res, ref, C.float())
    torch.cuda.synchronize()
    return out


base = run_all(False)
tuned = run_all(True)
for key, (sol, res, ref, Cf) in tuned.items():
    _, bres, _, _ = base[key]
    for form, t in res.items():
        r = ref + Cf if form.startswith("addmm") else ref
        scale = float(r.abs().max())
        rec = {"shape": "%s_%d_%d_%d" % key, "solution": sol, "form": form,
               "finite": bool(torch.isfinite(t).all()), "nonfinite": int((~torch.isfinite(t)).sum()),
               "max_err_vs_fp32": float((t.float() - r).abs().max() / scale),
               "default_finite": bool(torch.isfinite(bres[form]).all()),
               "default_max_err_vs_fp32": float((bres[form].float() - r).abs().max() / scale),
               "equal_to_default": bool(torch.equal(t, bres[form]))}
        print(json.dumps(rec), flush=True)
