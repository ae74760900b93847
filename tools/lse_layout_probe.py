import torch
for bounds in ([0, 2048, 4096], [0, 1, 37, 300, 531, 1024, 1151], [0, 8192, 16384]):
    T = bounds[-1]; H = 12; D = 128
    q = torch.randn((T, H, D), device="cuda").to(torch.bfloat16)
    cu = torch.tensor(bounds, dtype=torch.int32, device="cuda")
    mx = max(b - a for a, b in zip(bounds[:-1], bounds[1:]))
    out, lse, *_ = torch.ops.aten._flash_attention_forward(q, q, q, cu, cu, mx, mx, 0.0, True, False)
    # reference lse for head 0, last token of sequence 0
    a, b = bounds[0], bounds[1]
    s = (q[a:b, 0].float() @ q[a:b, 0].float().T) * D ** -0.5
    s = s.masked_fill(torch.ones_like(s, dtype=torch.bool).triu(1), float("-inf"))
    ref = torch.logsumexp(s, -1)
    print(bounds, "lse", tuple(lse.shape), lse.stride(), lse.dtype, "ref0", float(ref[-1]), "flat[h0]", float(lse.reshape(-1)[b - 1]))
