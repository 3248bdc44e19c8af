"""One small training step; saves every parameter gradient (tools/lnpack_eq.py)."""
import sys, torch
sys.path.insert(0, "conformer-nemo_amd")
from nemo.collections.asr.losses import CTCLoss
from nemo.collections.asr.modules import ConformerEncoder, ConvASRDecoder
torch.manual_seed(0)
B, T, V, U = 8, 1000, 256, 60
enc = ConformerEncoder(feat_in=80, n_layers=3, d_model=512, n_heads=8, dropout=0.1, dropout_emb=0.0, dropout_att=0.1).cuda().train()
dec = ConvASRDecoder(feat_in=512, num_classes=V).cuda().train()
loss_fn = CTCLoss(num_classes=V, zero_infinity=True, reduction="mean_batch")
g = torch.Generator(device="cuda").manual_seed(11)
x = torch.randn(B, 80, T, device="cuda", generator=g)
ln = torch.full((B,), T, dtype=torch.int64, device="cuda"); ln[1::4] = 731
tg = torch.randint(0, V, (B, U), device="cuda", generator=g)
tl = torch.full((B,), U, dtype=torch.int64, device="cuda")
torch.manual_seed(1234)
y, yl = enc(audio_signal=x, length=ln)
loss = loss_fn(log_probs=dec(encoder_output=y), targets=tg, input_lengths=yl, target_lengths=tl)
loss.backward()
torch.save({n: p.grad.detach().cpu() for n, p in list(enc.named_parameters()) + list(dec.named_parameters())}, sys.argv[1])
print("loss", float(loss))
