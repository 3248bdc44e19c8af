"""Golden fixtures for the RNN-T prediction network and greedy batch decoding
(include/cfm_rnnt_decode.h), from the REFERENCE modules run in float32 on the CPU:
  RNNTDecoder.predict / forward            nemo/collections/asr/modules/rnnt.py:50-283
  GreedyBatchedRNNTInfer (blank_as_pad)    nemo/collections/asr/parts/submodules/rnnt_greedy_decoding.py:365-616
  GreedyRNNTInfer (per utterance)          rnnt_greedy_decoding.py:191-362
Only where /root/reference exists:

    python tests/golden/gen_rnnt_decode_goldens.py   # writes tests/golden/rnnt_decode_*.npz

Loaded with gen_joint_goldens.py's typing-only shims (+ `Typing`, `HypothesisType`, and
`NeuralModule.as_frozen` as a null context: it only toggles requires_grad), none of which touches the arithmetic.  On the CPU the
reference log-softmaxes the joint output before the argmax (rnnt_greedy_decoding.py:184-185), so its
hypothesis scores are sums of log-probabilities; tokens, timesteps and final states do not depend
on that.  Weights are seeded uniform(-s, s) with the embedding's padding (blank) row kept at zero.
"""
import importlib.util
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_goldens import REF  # noqa: E402
from gen_joint_goldens import load_joint  # noqa: E402


def load_greedy():
    rnnt = load_joint()
    nt = sys.modules["nemo.core.neural_types"]
    nt.HypothesisType = lambda *a, **kw: None
    cls = sys.modules["nemo.core.classes"]

    class Typing:
        pass

    cls.Typing = Typing
    # NeuralModule.as_frozen (nemo/core/classes/module.py) only toggles requires_grad
    import contextlib
    for c in (rnnt.RNNTDecoder, rnnt.RNNTJoint):
        c.as_frozen = lambda self: contextlib.nullcontext()
    path = f"{REF}/nemo/collections/asr/parts/submodules/rnnt_greedy_decoding.py"
    spec = importlib.util.spec_from_file_location("rnnt_greedy_decoding_ref", path)
    gd = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gd)
    return rnnt, gd


CASES = {
    # name: (V (no blank), pred_hidden, layers, enc_hidden, joint_hidden, activation, B, T, lens, U, max_symbols,
    #        weight scale, enc scale, blank logit bias, seed) -- the blank bias mixes blank and label emissions
    "rnnt_decode_small": (12, 16, 1, 20, 24, "relu", 3, 9, [9, 6, 1], 4, 3, 0.5, 1.0, 2.0, 1),
    "rnnt_decode_2layer": (30, 32, 2, 24, 40, "tanh", 4, 12, [12, 11, 7, 0], 6, 2, 0.35, 1.5, 2.0, 2),
    "rnnt_decode_wide": (100, 64, 1, 48, 64, "relu", 2, 20, [20, 13], 8, 5, 0.25, 2.0, 3.0, 3),
    # mostly blank: whole early frames emit nothing (the reference's `hidden is None` path)
    "rnnt_decode_sparse": (12, 16, 1, 20, 24, "relu", 3, 15, [15, 15, 10], 4, 3, 0.5, 1.0, 3.5, 5),
}


def main():
    rnnt, gd = load_greedy()
    for name, (V, H, L, D1, J, act, B, T, lens, U, ms, ws, es, bb, seed) in CASES.items():
        torch.manual_seed(seed)
        dec = rnnt.RNNTDecoder(prednet=dict(pred_hidden=H, pred_rnn_layers=L), vocab_size=V).eval()
        joint = rnnt.RNNTJoint(jointnet=dict(encoder_hidden=D1, pred_hidden=H, joint_hidden=J, activation=act),
                               num_classes=V).eval()
        with torch.no_grad():
            for p in list(dec.parameters()) + list(joint.parameters()):
                p.uniform_(-ws, ws)
            dec.prediction["embed"].weight[V].zero_()        # padding_idx = blank
            joint.joint_net[-1].bias[V] += bb
        g = np.random.default_rng(seed)
        enc = torch.tensor(g.standard_normal((B, D1, T)) * es, dtype=torch.float32)
        enc_len = torch.tensor(lens, dtype=torch.int64)
        y = torch.tensor(g.integers(0, V, (B, U)), dtype=torch.int64)
        out = {"V": np.int64(V), "H": np.int64(H), "L": np.int64(L), "D1": np.int64(D1), "J": np.int64(J),
               "activation": np.array(act), "max_symbols": np.int64(ms), "enc": enc.numpy(),
               "enc_len": enc_len.numpy(), "y": y.numpy()}
        for k, v in dec.state_dict().items():
            out["dec/" + k] = v.numpy()
        for k, v in joint.state_dict().items():
            out["joint/" + k] = v.numpy()
        with torch.no_grad():
            # teacher-forced prediction network (RNNTDecoder.forward -> predict(add_sos=True))
            gout, _, st = dec(targets=y, target_length=torch.full((B,), U))
            out["pred_g"] = gout.numpy()                       # (B, H, U + 1)
            out["pred_h"], out["pred_c"] = st[0].numpy(), st[1].numpy()
            # with an initial state, no SOS
            h0 = torch.tensor(g.standard_normal((L, B, H)) * 0.5, dtype=torch.float32)
            c0 = torch.tensor(g.standard_normal((L, B, H)) * 0.5, dtype=torch.float32)
            g2, st2 = dec.predict(y, state=[h0, c0], add_sos=False)
            out.update(h0=h0.numpy(), c0=c0.numpy(), pred2_g=g2.numpy(), pred2_h=st2[0].numpy(),
                       pred2_c=st2[1].numpy())
            greedy = gd.GreedyBatchedRNNTInfer(dec, joint, blank_index=V, max_symbols_per_step=ms)
            hyps = greedy(encoder_output=enc, encoded_lengths=enc_len)[0]
            single = gd.GreedyRNNTInfer(dec, joint, blank_index=V, max_symbols_per_step=ms)
            hyps1 = single(encoder_output=enc, encoded_lengths=enc_len)[0]
        ntok = [len(h.y_sequence) for h in hyps]
        tok = np.full((B, max(1, max(ntok))), -1, np.int64)
        tst = np.full_like(tok, -1)
        for b, h in enumerate(hyps):
            tok[b, :ntok[b]] = h.y_sequence.numpy()
            tst[b, :ntok[b]] = np.array(h.timestep, dtype=np.int64)
            h1 = hyps1[b]
            assert h1.y_sequence.tolist() == h.y_sequence.tolist(), "batched and per-utterance greedy differ"
        out.update(tokens=tok, timesteps=tst, ntok=np.array(ntok), scores=np.array([h.score for h in hyps]))
        has_state = hyps[0].dec_state is not None
        out["has_state"] = np.int64(has_state)
        if has_state:
            out["final_h"] = np.stack([np.stack([s.numpy() for s in h.dec_state[0]]) for h in hyps], 1)
            out["final_c"] = np.stack([np.stack([s.numpy() for s in h.dec_state[1]]) for h in hyps], 1)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        print(name, "tokens per utterance", ntok, "max per step", ms)


if __name__ == "__main__":
    main()
