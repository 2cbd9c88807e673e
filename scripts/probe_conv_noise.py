import sys, torch
sys.path.insert(0, '/root/repo')
from distributedauc_amd.backbone import build_backbone
from distributedauc_amd import conv1x1 as C
dev = torch.device('cuda', 0)
for seed in range(4):
    torch.manual_seed(seed)
    base = build_backbone("resnet50", num_classes=2)
    x = torch.randn(8, 3, 64, 64, device=dev).contiguous(memory_format=torch.channels_last)
    runs = {}
    for name, amp, fbn, fg in (("fp32", False, False, False), ("bf16", True, False, False), ("fast", True, True, True), ("bn", True, True, False), ("gemm", True, False, True)):
        net = build_backbone("resnet50", num_classes=2)
        net.load_state_dict(base.state_dict())
        net = net.to(dev).to(memory_format=torch.channels_last).train()
        net.set_fused_bn(fbn).set_gemm_conv1x1(fg)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = net(x)
        runs[name] = out.detach().float()
    r = runs["fp32"]
    print(seed, "scale", float(r.abs().max()), {k: round(float((v - r).abs().max()), 4) for k, v in runs.items() if k != "fp32"}, flush=True)
