"""Probe: ResNet-50 1x1 convolutions (channels-last bf16, batch 256) as MIOpen convs vs plain GEMMs.

For every distinct stride-1 1x1 conv shape: forward + backward (data + weight) time through
F.conv2d (MIOpen) and through torch.mm on the [M, C] views (hipBLASLt), HIP events, median.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

dev = torch.device("cuda", 0)
B = 256
SHAPES = [  # (H, Cin, Cout, count in ResNet-50)
    (56, 64, 64, 1), (56, 256, 64, 2), (56, 64, 256, 4), (56, 256, 128, 1),
    (28, 512, 128, 3), (28, 128, 512, 4), (28, 512, 256, 1),
    (14, 1024, 256, 5), (14, 256, 1024, 6), (14, 1024, 512, 1),
    (7, 2048, 512, 2), (7, 512, 2048, 3),
]


def timeit(fn, reps=20, warm=5):
    for _ in range(warm):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2] * 1e3


tot_conv = tot_mm = 0.0
for H, cin, cout, cnt in SHAPES:
    x = torch.randn(B, cin, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(cout, cin, 1, 1, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(B, cout, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    M = B * H * H

    def conv_fb():
        xx = x.detach().requires_grad_(True)
        ww = w.detach().requires_grad_(True)
        y = F.conv2d(xx, ww)
        y.backward(gy)

    x2 = x.permute(0, 2, 3, 1).reshape(M, cin)
    g2 = gy.permute(0, 2, 3, 1).reshape(M, cout)
    w2 = w.reshape(cout, cin)

    def mm_fb():
        y = torch.mm(x2, w2.t())
        dx = torch.mm(g2, w2)
        dw = torch.mm(g2.t(), x2)
        return y, dx, dw

    # per direction: MIOpen via aten.convolution_backward, GEMMs via torch.mm (dW split-K over 16 slabs)
    xx, ww = x.detach(), w.detach()
    t_cf = timeit(lambda: F.conv2d(xx, ww))
    t_cd = timeit(lambda: torch.ops.aten.convolution_backward(gy, xx, ww, None, [1, 1], [0, 0], [1, 1], False,
                                                             [0, 0], 1, [True, False, False]))
    t_cw = timeit(lambda: torch.ops.aten.convolution_backward(gy, xx, ww, None, [1, 1], [0, 0], [1, 1], False,
                                                             [0, 0], 1, [False, True, False]))
    t_mf = timeit(lambda: torch.mm(x2, w2.t()))
    t_md = timeit(lambda: torch.mm(g2, w2))
    S = 16 if M % 16 == 0 else 1
    t_mw = timeit(lambda: torch.bmm(g2.view(S, M // S, cout).transpose(1, 2), x2.view(S, M // S, cin)).sum(0))
    tc = t_cf + t_cd + t_cw
    tm = min(t_cf, t_mf) + min(t_cd, t_md) + min(t_cw, t_mw)
    tot_conv += tc * cnt
    tot_mm += tm * cnt
    print(f"H={H:3d} {cin:5d}->{cout:5d} x{cnt}: fwd conv {t_cf:7.1f} mm {t_mf:7.1f} | dgrad conv {t_cd:7.1f} "
          f"mm {t_md:7.1f} | wgrad conv {t_cw:7.1f} mm(splitK) {t_mw:7.1f} us", flush=True)
print(f"TOTAL 1x1 stride-1 per step: MIOpen {tot_conv / 1e3:.2f} ms  best-of-each {tot_mm / 1e3:.2f} ms", flush=True)
