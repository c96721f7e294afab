import torch
M=30720
for (K,N) in ((1024,512),(1024,4096),(512,4096),(4096,1024)):
    a=torch.randn(M,K,device='cuda',dtype=torch.bfloat16); b=torch.randn(K,N,device='cuda',dtype=torch.bfloat16)
    for _ in range(5): c=torch.matmul(a,b)
    try:
        for _ in range(5): c=torch.mm(a,b,out_dtype=torch.float32)
        print("mm out_dtype f32 ok", c.dtype)
    except Exception as e:
        print("out_dtype err", str(e)[:100])
torch.cuda.synchronize()
