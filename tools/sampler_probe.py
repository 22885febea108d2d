import sys, torch, time
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from theroundtaible_amd import ops
DEV='cuda'
def t(fn, n=20):
    fn(); torch.cuda.synchronize()
    a=torch.cuda.Event(enable_timing=True); b=torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b)*1000/n
for V in (32000, 128256):
  for B in (1, 3):
    lg=(torch.randn(B,V,device=DEV)).to(torch.bfloat16)
    ws=ops.sample_workspace(B, DEV); out=torch.empty(B,dtype=torch.int64,device=DEV)
    s=torch.arange(B,device=DEV); o=torch.zeros(B,dtype=torch.int64,device=DEV)
    T=torch.full((B,),0.8,device=DEV); one=torch.ones(B,device=DEV); k0=torch.zeros(B,dtype=torch.int32,device=DEV)
    for name,(temp,p,k) in {'greedy':(T*0,one,k0),'unfilt':(T,one,k0),'topp.9':(T,one*0.9,k0),'topp.3':(T,one*0.3,k0),
                            'topk40':(T,one,k0+40),'topk40p.9':(T,one*0.9,k0+40),'topk64':(T,one,k0+64),'topk4000':(T,one,k0+4000)}.items():
        print(V,B,name, round(t(lambda: ops.sample(lg,temp,p,k,s,o,out,ws=ws)),1))
# per-row view of the B=3 top-p launches (fixed seeds: each row takes the same path every call)
V = 128256
lg = torch.randn(3, V, device=DEV).to(torch.bfloat16)
for p_ in (0.9, 0.3):
    for b in range(3):
        ws = ops.sample_workspace(1, DEV); out = torch.empty(1, dtype=torch.int64, device=DEV)
        s = torch.tensor([b], device=DEV); o = torch.zeros(1, dtype=torch.int64, device=DEV)
        T = torch.full((1,), 0.8, device=DEV); P = torch.full((1,), p_, device=DEV)
        k0 = torch.zeros(1, dtype=torch.int32, device=DEV)
        print("row", b, "topp", p_, round(t(lambda: ops.sample(lg[b:b + 1], T, P, k0, s, o, out, ws=ws)), 1))
