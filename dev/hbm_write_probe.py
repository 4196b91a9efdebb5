import torch, time
x = torch.empty(346 * 1024 * 1024 // 2, dtype=torch.bfloat16, device="cuda")
y = torch.empty_like(x)
for f in (lambda: x.fill_(1.0), lambda: y.copy_(x)):
    for _ in range(3): f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): f()
    e1.record(); e1.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"{ms*1e3:.1f} us  {x.numel()*2/ms/1e9:.2f} TB/s (per direction)")
