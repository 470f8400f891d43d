import torch,time
d='cuda'
for (M,K,N) in [(4194304,1152,128),(8192,8192,8192),(1048576,2304,256)]:
    a=torch.randn(M,K,device=d).bfloat16(); b=torch.randn(K,N,device=d).bfloat16()
    for _ in range(3): c=a@b
    torch.cuda.synchronize(); e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): c=a@b
    e1.record(); torch.cuda.synchronize(); ms=e0.elapsed_time(e1)/10
    print(M,K,N, ms, 2*M*K*N/ms/1e9, "TF/s")
