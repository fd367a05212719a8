import torch
def t(fn, it=30):
    for _ in range(3): fn()
    e0,e1=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1)/it*1e3
for n,fin in [(169343,128),(232965,602),(44906,50)]:
    x=torch.randn(n,fin,device='cuda'); w=torch.randn(64,fin,device='cuda'); b=torch.randn(64,device='cuda')
    print(n,fin,'mm',round(t(lambda: torch.mm(x,w.t())),1),'addmm',round(t(lambda: torch.addmm(b,x,w.t())),1))
