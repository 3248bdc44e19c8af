"""GPU parity of the RNN-T prediction network and greedy decoding (include/cfm_rnnt_decode.h) against
the REFERENCE modules' outputs (tests/golden/rnnt_decode_*.npz, gen_rnnt_decode_goldens.py) and the
float64 oracle (oracle/rnnt_decode_oracle.py).  Gates: fp32 LSTM outputs / states rtol 1e-4; greedy
tokens and timesteps exact; scores within 1e-4 relative."""
import glob
import os

import numpy as np
import pytest
import torch

import rnnt_decode_oracle as RD

pytestmark = pytest.mark.gpu
FILES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "rnnt_decode_*.npz")))
IDS = [os.path.basename(f)[:-4] for f in FILES]


def _modules(z):
    from nemo.collections.asr.modules import RNNTDecoder, RNNTJoint
    V, H, L = int(z["V"]), int(z["H"]), int(z["L"])
    dec = RNNTDecoder(prednet=dict(pred_hidden=H, pred_rnn_layers=L), vocab_size=V)
    joint = RNNTJoint(jointnet=dict(encoder_hidden=int(z["D1"]), pred_hidden=H, joint_hidden=int(z["J"]),
                                    activation=str(z["activation"])), num_classes=V)
    dec.load_state_dict({k[4:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("dec/")})
    joint.load_state_dict({k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("joint/")})
    return dec.cuda().eval(), joint.cuda().eval()


@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_prediction_network_matches_reference(path):
    z = np.load(path)
    dec, _ = _modules(z)
    y = torch.from_numpy(z["y"]).cuda()
    with torch.no_grad():
        g, ln, st = dec(targets=y, target_length=torch.full((y.shape[0],), y.shape[1]))
        np.testing.assert_allclose(g.cpu().numpy(), z["pred_g"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(st[0].cpu().numpy(), z["pred_h"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(st[1].cpu().numpy(), z["pred_c"], rtol=1e-4, atol=1e-5)
        g2, st2 = dec.predict(y, state=[torch.from_numpy(z["h0"]).cuda(), torch.from_numpy(z["c0"]).cuda()],
                              add_sos=False)
        np.testing.assert_allclose(g2.cpu().numpy(), z["pred2_g"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(st2[1].cpu().numpy(), z["pred2_c"], rtol=1e-4, atol=1e-5)
        # y=None: one zero step (the greedy decoder's SOS call), with and without add_sos
        g3, _ = dec.predict(None, state=None, add_sos=False, batch_size=3)
        g4, _ = dec.predict(None, state=None, add_sos=True, batch_size=3)
        assert g3.shape == (3, 1, int(z["H"])) and g4.shape == (3, 2, int(z["H"]))
        torch.testing.assert_close(g4[:, :1], g3)


def _check_hyps(hyps, z, scores_from_ref):
    for b, h in enumerate(hyps):
        n = int(z["ntok"][b])
        assert h.y_sequence.tolist() == z["tokens"][b, :n].tolist(), b
        assert list(h.timestep) == z["timesteps"][b, :n].tolist(), b
        if scores_from_ref:
            assert abs(h.score - z["scores"][b]) <= 1e-4 * max(1.0, abs(z["scores"][b])), (h.score, z["scores"][b])
        assert int(h.length) == int(z["enc_len"][b])


@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_greedy_batched_matches_reference(path):
    from nemo.collections.asr.parts.submodules.rnnt_greedy_decoding import GreedyBatchedRNNTInfer, GreedyRNNTInfer
    z = np.load(path)
    dec, joint = _modules(z)
    V = int(z["V"])
    enc = torch.from_numpy(z["enc"]).cuda()
    ln = torch.from_numpy(z["enc_len"]).cuda()
    joint.log_softmax = True          # the CPU reference log-normalised: compare its scores directly
    hyps = GreedyBatchedRNNTInfer(dec, joint, blank_index=V, max_symbols_per_step=int(z["max_symbols"]))(
        encoder_output=enc, encoded_lengths=ln)[0]
    _check_hyps(hyps, z, True)
    if int(z["has_state"]):
        for b, h in enumerate(hyps):
            np.testing.assert_allclose(torch.stack(list(h.dec_state[0])).numpy(), z["final_h"][:, b], rtol=1e-4,
                                       atol=1e-5)
            np.testing.assert_allclose(torch.stack(list(h.dec_state[1])).numpy(), z["final_c"][:, b], rtol=1e-4,
                                       atol=1e-5)
    else:
        assert all(h.dec_state is None for h in hyps)
    hyps1 = GreedyRNNTInfer(dec, joint, blank_index=V, max_symbols_per_step=int(z["max_symbols"]))(
        encoder_output=enc, encoded_lengths=ln)[0]
    _check_hyps(hyps1, z, True)
    # GPU semantics (joint.log_softmax None): raw-logit scores, against the oracle
    joint.log_softmax = None
    hyps2 = GreedyBatchedRNNTInfer(dec, joint, blank_index=V, max_symbols_per_step=int(z["max_symbols"]))(
        encoder_output=enc, encoded_lengths=ln)[0]
    d = {k[4:]: z[k] for k in z.files if k.startswith("dec/")}
    j = {k[6:]: z[k] for k in z.files if k.startswith("joint/")}
    res, _ = RD.greedy_decode(d, j, int(z["L"]), str(z["activation"]), z["enc"], z["enc_len"], V,
                              int(z["max_symbols"]), log_normalize=False)
    for h, (toks, _, score, _, _) in zip(hyps2, res):
        assert h.y_sequence.tolist() == toks
        assert abs(h.score - score) <= 1e-4 * max(1.0, abs(score))


def test_transducer_large_shapes_against_oracle():
    """conformer_transducer_bpe.yaml shapes (pred_hidden 640, joint_hidden 640, d_model 512, V=1024,
    max_symbols 30) on a short ragged batch, against the float64 oracle; plus batch invariance."""
    from nemo.collections.asr.modules import RNNTDecoder, RNNTJoint
    from nemo.collections.asr.parts.submodules.rnnt_greedy_decoding import GreedyBatchedRNNTInfer
    torch.manual_seed(0)
    V, H, J, D1, B, T = 1024, 640, 640, 512, 4, 48
    dec = RNNTDecoder(prednet=dict(pred_hidden=H, pred_rnn_layers=1), vocab_size=V)
    joint = RNNTJoint(jointnet=dict(encoder_hidden=D1, pred_hidden=H, joint_hidden=J, activation="relu"),
                      num_classes=V)
    with torch.no_grad():
        for p in list(dec.parameters()) + list(joint.parameters()):
            p.uniform_(-0.08, 0.08)
        dec.prediction["embed"].weight[V].zero_()
        joint.joint_net[-1].bias[V] += 0.6
    dec, joint = dec.cuda().eval(), joint.cuda().eval()
    enc = torch.randn(B, D1, T, device="cuda")
    ln = torch.tensor([48, 40, 17, 1], device="cuda")
    greedy = GreedyBatchedRNNTInfer(dec, joint, blank_index=V, max_symbols_per_step=30)
    hyps = greedy(encoder_output=enc, encoded_lengths=ln)[0]
    d = {k: v.cpu().numpy() for k, v in dec.state_dict().items()}
    j = {k: v.cpu().numpy() for k, v in joint.state_dict().items()}
    res, _ = RD.greedy_decode(d, j, 1, "relu", enc.cpu().numpy(), ln.cpu().numpy(), V, 30)
    ntoks = [len(r[0]) for r in res]
    assert sum(ntoks) > 10 and any(len(r[0]) < ln[i].item() * 30 for i, r in enumerate(res))   # mixed emissions
    for h, (toks, steps, score, hh, cc) in zip(hyps, res):
        assert h.y_sequence.tolist() == toks and list(h.timestep) == steps
        assert abs(h.score - score) <= 1e-4 * max(1.0, abs(score))
    # an utterance decodes the same alone as inside the batch
    solo = greedy(encoder_output=enc[2:3].contiguous(), encoded_lengths=ln[2:3])[0][0]
    assert solo.y_sequence.tolist() == hyps[2].y_sequence.tolist()


def test_cpu_is_refused_and_zero_length():
    from nemo.collections.asr.modules import RNNTDecoder
    dec = RNNTDecoder(prednet=dict(pred_hidden=16, pred_rnn_layers=1), vocab_size=5)
    with pytest.raises(RuntimeError):
        dec.predict(torch.zeros(1, 2, dtype=torch.long))
    dec = dec.cuda().eval()
    with pytest.raises(IndexError):
        with torch.no_grad():
            dec.predict(torch.full((1, 2), 9, dtype=torch.long, device="cuda"))
