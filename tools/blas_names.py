import torch, torch.nn.functional as F
for (M,N,K) in [(32768,768,3072),(32768,768,768),(32768,3072,768),(32768,2304,768)]:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16); w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(3): F.linear(x, w)
    torch.cuda.synchronize()
