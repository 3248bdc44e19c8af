"""Attention backward at the BASELINE config-3 shape (B=32, T'=250, H=8, dk=64, bf16): times
cfm_op_rel_attention_backward with the fused score producer on and off (CFM_ATTN_BWD_FUSED, read
once per process, so each arm runs in its own child) and checks the two arms agree.
Usage: python tools/attn_bwd_bench.py [B T H dk]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(B, T, H, dk, out):
    sys.path.insert(0, os.path.join(ROOT, "conformer-nemo_amd"))
    import numpy as np
    import torch
    from conformer_amd import _lib
    lib = _lib.load()
    d = H * dk
    M = B * T
    g = torch.Generator().manual_seed(0)
    q, k, v = (torch.randn(M, d, generator=g).bfloat16().cuda() for _ in range(3))
    p = torch.randn(2 * T - 1, d, generator=g).bfloat16().cuda()
    u, vb = (0.1 * torch.randn(d, generator=g)).cuda(), (0.1 * torch.randn(d, generator=g)).cuda()
    dctx = torch.randn(M, d, generator=g).cuda()
    lens = torch.tensor([T - (7 * b) % (T // 3) for b in range(B)], dtype=torch.int32).cuda()
    dq, dkey, dv = (torch.empty(M, d, device="cuda") for _ in range(3))
    dp = torch.empty(2 * T - 1, d, device="cuda")
    du, dvb = torch.empty(d, device="cuda"), torch.empty(d, device="cuda")
    n = lib.cfm_op_rel_attention_backward_ws_size(1, B, T, H, dk)
    ws = torch.empty(n, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def run():
        _lib.check(lib.cfm_op_rel_attention_backward(1, q.data_ptr(), k.data_ptr(), v.data_ptr(), p.data_ptr(),
                                                     u.data_ptr(), vb.data_ptr(), lens.data_ptr(), B, T, H, dk, -1,
                                                     -1, dctx.data_ptr(), dq.data_ptr(), dkey.data_ptr(),
                                                     dv.data_ptr(), dp.data_ptr(), du.data_ptr(), dvb.data_ptr(),
                                                     ws.data_ptr(), n, st), "rel_attention_backward")
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record()
    torch.cuda.synchronize()
    np.savez(out, us=e0.elapsed_time(e1) / 20 * 1e3, dq=dq.cpu().numpy(), dk=dkey.cpu().numpy(),
             dv=dv.cpu().numpy(), dp=dp.cpu().numpy(), du=du.cpu().numpy(), dvb=dvb.cpu().numpy())


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(*map(int, sys.argv[2:6]), sys.argv[6])
        return
    import numpy as np
    shape = list(map(int, sys.argv[1:5])) if len(sys.argv) >= 5 else [32, 250, 8, 64]
    import tempfile
    tmp = tempfile.mkdtemp()
    res = {}
    for arm in ("0", "1"):
        out = os.path.join(tmp, f"attn_bwd_{arm}.npz")
        env = dict(os.environ, CFM_ATTN_BWD_FUSED=arm)
        subprocess.run([sys.executable, __file__, "--child", *map(str, shape), out], env=env, check=True, timeout=300)
        res[arm] = np.load(out)
    print(f"shape B,T,H,dk={shape}: materialised {float(res['0']['us']):.1f} us, fused {float(res['1']['us']):.1f} us")
    for name in ("dq", "dk", "dv", "dp", "du", "dvb"):
        a, b = res["0"][name].astype(np.float64), res["1"][name].astype(np.float64)
        print(f"  {name}: relL2(fused vs materialised) = {np.linalg.norm(a - b) / max(np.linalg.norm(a), 1e-30):.2e}")


if __name__ == "__main__":
    main()
