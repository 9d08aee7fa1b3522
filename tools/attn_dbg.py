import sys, torch
sys.path.insert(0, 'multimodal-embedding_amd'); sys.path.insert(0, 'tests')
from mme import ops
from test_gpu_kernels import attn_ref
for (B,T,H,hd) in [(1,16,1,80),(1,16,1,72),(1,64,1,80),(1,17,1,80),(1,40,2,80)]:
    torch.manual_seed(0)
    qkv = torch.randn(B*T, 3*H*hd, device='cuda').to(torch.bfloat16)
    out = ops.attention(qkv, B, T, H, hd)
    ref = attn_ref(qkv, B, T, H, hd, None, False, hd**-0.5)
    err = (out.float()-ref).abs()
    print(B,T,H,hd, 'max err', err.max().item(), 'err by row', [round(x,2) for x in err.max(1).values.tolist()][:20])
    print('   err by col>64', err[:, :64].max().item(), err[:, 64:].max().item())
    # zero the tail dims of q/k to see whether the K16 step is the culprit
    q2 = qkv.clone().view(B*T, 3, H, hd); q2[:, :2, :, 64:] = 0; q2 = q2.view(B*T, -1)
    out2 = ops.attention(q2, B, T, H, hd); ref2 = attn_ref(q2, B, T, H, hd, None, False, hd**-0.5)
    print('   with q/k dims>=64 zeroed:', (out2.float()-ref2).abs().max().item())
