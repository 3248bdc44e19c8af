"""Golden fixtures for on-device spectrogram augmentation (include/cfm_augment.h), from
the REFERENCE modules (nemo/collections/asr/parts/submodules/spectr_augment.py and
SpectrogramAugmentation in nemo/collections/asr/modules/audio_preprocessing.py:416-521).  Only where
/root/reference exists:

    python tests/golden/gen_augment_goldens.py   # writes tests/golden/augment_*.npz

spectr_augment.py imports `nemo.core.classes.{Typing, typecheck}` and four neural-type names; they
are shimmed with typing-only stand-ins (typecheck as a no-op decorator), which do not touch the
masking arithmetic or the random.Random call sequence.  SpectrogramAugmentation's class body is
taken from audio_preprocessing.py by source slicing (the file's other imports pull in torchaudio /
librosa, which are absent) and executed in a namespace holding the shimmed spectr_augment classes.

Per case: input spec (B, F, T) fp32, lengths, the rng seed, the module kwargs, and the reference
output.  SpecShot draws from torch's CPU generator, so only its kept fraction is recorded.
"""
import importlib.util
import json
import os
import random
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _shims():
    class typecheck:
        def __init__(self, *a, **k):
            pass

        def __call__(self, f):
            return f

    class Typing:
        pass

    core = types.ModuleType("nemo.core.classes")
    core.Typing, core.typecheck = Typing, typecheck
    nt = types.ModuleType("nemo.core.neural_types")
    for k in ("LengthsType", "NeuralType", "SpectrogramType"):
        setattr(nt, k, lambda *a, **kw: None)
    for name in ("nemo", "nemo.core"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["nemo.core.classes"] = core
    sys.modules["nemo.core.neural_types"] = nt


def load_reference():
    _shims()
    path = f"{REF}/nemo/collections/asr/parts/submodules/spectr_augment.py"
    spec = importlib.util.spec_from_file_location("spectr_augment_ref", path)
    sa = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sa)
    src = open(f"{REF}/nemo/collections/asr/modules/audio_preprocessing.py").read()
    i = src.index("class SpectrogramAugmentation(")
    j = src.index("class MaskedPatchAugmentation(")
    ns = dict(torch=torch, random=random, nn=torch.nn, NeuralModule=torch.nn.Module, typecheck=sys.modules[
        "nemo.core.classes"].typecheck, NeuralType=lambda *a, **k: None, SpectrogramType=lambda *a, **k: None,
        LengthsType=lambda *a, **k: None, SpecAugment=sa.SpecAugment, SpecCutout=sa.SpecCutout,
        SpecShot=sa.SpecShot)
    exec(compile(src[i:j], "audio_preprocessing.py[SpectrogramAugmentation]", "exec"), ns)
    return sa, ns["SpectrogramAugmentation"]


CASES = {
    # name: (module, kwargs, B, F, T, lengths, seed)
    # conformer_ctc_bpe.yaml:94-100 spec_augment block (freq 2 x 27, time 10 x 0.05 adaptive)
    "augment_ctc_bpe": ("SpecAugment", dict(freq_masks=2, time_masks=10, freq_width=27, time_width=0.05),
                        4, 80, 1008, [1000, 997, 641, 123], 11),
    "augment_int_width": ("SpecAugment", dict(freq_masks=3, time_masks=4, freq_width=10, time_width=25,
                                              mask_value=-1.5), 3, 64, 160, [160, 77, 9], 12),
    "augment_cutout": ("SpecCutout", dict(rect_masks=5, rect_time=25, rect_freq=20), 3, 80, 200, None, 13),
    "augment_choice": ("SpectrogramAugmentation", dict(freq_masks=2, time_masks=5, freq_width=15, time_width=0.1,
                                                       rect_masks=3, rect_time=12, rect_freq=9), 2, 80, 300,
                       [300, 211], 14),
}


def main():
    sa, SpectrogramAugmentation = load_reference()
    for name, (kind, kw, B, F, T, lens, seed) in CASES.items():
        g = np.random.default_rng(seed)
        x = g.standard_normal((B, F, T)).astype(np.float32)
        ln = np.array(lens if lens is not None else [T] * B, dtype=np.int64)
        spec = torch.from_numpy(x.copy())
        length = torch.from_numpy(ln)
        if kind == "SpectrogramAugmentation":
            random.seed(seed)   # the module's random.choice uses the global generator
            m = SpectrogramAugmentation(rng=random.Random(seed), **kw)
            outs = []
            for _ in range(6):   # several calls so both augment types are drawn
                s = torch.from_numpy(x.copy())
                outs.append(m(input_spec=s, length=length).numpy())
            y = np.stack(outs)
        else:
            m = getattr(sa, kind)(rng=random.Random(seed), **kw)
            y = (m(input_spec=spec, length=length) if kind == "SpecAugment" else m(input_spec=spec)).numpy()
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), x=x, lengths=ln, seed=np.int64(seed),
                            kind=np.array(kind), kwargs_json=np.array(json.dumps(kw)), y=y)
        print(name, kind, y.shape, "masked fraction", float((y != np.broadcast_to(x, y.shape)).mean()))
    # SpecShot: kept fraction only (torch CPU generator, not reproduced on the device)
    torch.manual_seed(0)
    s = sa.SpecShot(mask_ratio=0.3)(input_spec=torch.ones(8, 80, 500))
    np.savez_compressed(os.path.join(HERE, "augment_specshot.npz"), mask_ratio=np.float64(0.3),
                        kept=np.float64(float(s.mean())))
    print("specshot kept", float(s.mean()))


if __name__ == "__main__":
    main()
