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
# the captured step's form: sampler + decode-step bookkeeping in one launch (B = 3, V = 128K,
# hidden 4096 embedding row copy), timed over replays of a captured graph
B, V, H, bs, maxb = 3, 128256, 4096, 32, 64
lg = torch.randn(B, V, device=DEV).to(torch.bfloat16)
embed = torch.randn(V, H, device=DEV).to(torch.bfloat16)
bt = torch.arange(B * maxb, device=DEV, dtype=torch.int32).reshape(B, maxb)
seeds = torch.arange(B, device=DEV, dtype=torch.int64)
pos = torch.full((B,), 100, dtype=torch.int64, device=DEV)
st = dict(out=torch.zeros(4096, B, dtype=torch.int64, device=DEV), ids=torch.zeros(B, dtype=torch.int64, device=DEV),
          pos=pos, ctx=(pos + 1).to(torch.int32), step=torch.zeros(1, dtype=torch.int64, device=DEV),
          slots=torch.zeros(B, dtype=torch.int64, device=DEV), offs=pos + 1,
          res=torch.zeros(B, H, dtype=torch.bfloat16, device=DEV))
ws = ops.sample_workspace(B, DEV)
nxt = torch.zeros(B, dtype=torch.int64, device=DEV)
for name, (temp, p, k) in {'greedy': (torch.zeros(B, device=DEV), torch.ones(B, device=DEV), torch.zeros(B, dtype=torch.int32, device=DEV)),
                           'topp.95': (torch.full((B,), 0.7, device=DEV), torch.full((B,), 0.95, device=DEV), torch.zeros(B, dtype=torch.int32, device=DEV))}.items():
    st["pos"].fill_(100); st["step"].zero_()
    def adv():
        ops.sample_advance(lg, temp, p, k, seeds, st["offs"], ws, nxt, st["out"], st["ids"], st["pos"], st["ctx"],
                           st["step"], st["slots"], st["res"], bt, embed, bs)
    adv(); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(20):
                adv()
    torch.cuda.synchronize()
    st["pos"].fill_(100)
    g.replay(); torch.cuda.synchronize()
    st["pos"].fill_(100)
    a_ = torch.cuda.Event(enable_timing=True); b_ = torch.cuda.Event(enable_timing=True)
    a_.record(); g.replay(); b_.record(); torch.cuda.synchronize()
    print("advance B=3", name, round(a_.elapsed_time(b_) * 1000 / 20, 1))
