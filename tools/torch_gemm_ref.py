# Reference point only (developer tool): torch.nn.functional.linear (hipBLASLt) on the encoder GEMM shapes.
import torch, time
torch.manual_seed(0)
M=206426
shapes={"qkv":(2304,768),"o":(768,768),"ffn1":(3072,768),"ffn2":(768,3072)}
for name,(N,K) in shapes.items():
    A=torch.randn(M,K,device="cuda",dtype=torch.bfloat16)
    W=torch.randn(N,K,device="cuda",dtype=torch.bfloat16)*0.02
    b=torch.randn(N,device="cuda",dtype=torch.bfloat16)
    for _ in range(3): y=torch.nn.functional.linear(A,W,b)
    torch.cuda.synchronize()
    t=time.perf_counter()
    for _ in range(10): y=torch.nn.functional.linear(A,W,b)
    torch.cuda.synchronize()
    ms=(time.perf_counter()-t)/10*1e3
    print(name, f"{ms:.3f} ms", f"{2*M*N*K/ms/1e9:.0f} TF")
