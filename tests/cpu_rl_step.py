"""TEST-ONLY torch-CPU stand-in for rl_step (the product rl_step runs the HIP kernel only).

Lets the data-parallel trainer loop, sentinel protocol and gradient sync be exercised with
gloo on CPU.  Same math as pipelinerl/finetune/rl/__init__.py:199-292 (ppo / reinforce, KL,
entropy, token weights, masked sums) on fp32 logits.
"""

import torch
import torch.nn.functional as F


def cpu_rl_step(model, batch, current_step, max_step, config):
    if batch.is_packed:
        from pipelinerl_amd.finetune.attention import packed_kwargs, uses_varlen

        extra = packed_kwargs(batch, batch.input_ids.device) if uses_varlen(model) else {}
        out = model(input_ids=batch.input_ids, position_ids=batch.position_ids, **extra)
    else:
        out = model(input_ids=batch.input_ids, attention_mask=batch.attention_mask)
    logits = out.logits[:, :-1].float() / config.temperature
    lp_all = F.log_softmax(logits, -1)
    ent = -(lp_all.exp() * lp_all).sum(-1)
    lp = torch.gather(lp_all, 2, batch.input_ids[:, 1:, None])[..., 0]
    mask = (batch.labels[:, 1:] != -100).float()
    old, ref, adv = batch.old_logprobs[:, 1:], batch.ref_logprobs[:, 1:], batch.advantages[:, 1:]
    w = torch.full_like(old, 1.0 / config.batch_size)
    ratio = torch.exp(lp - old)
    c = torch.clamp(ref - lp, -config.clamp_log_ratio_ref_new_value, config.clamp_log_ratio_ref_new_value)
    kl = torch.exp(c) - c - 1
    frac = current_step / max_step
    kl_c = config.kl_coef + (config.final_kl_coef - config.kl_coef) * frac
    ent_c = config.entropy_bonus + (config.final_entropy_bonus - config.entropy_bonus) * frac
    if config.policy_loss == "ppo":
        pol = torch.min(ratio * adv, torch.clamp(ratio, 1 - config.epsilon, 1 + config.epsilon) * adv)
        r_used = ratio
    else:
        r_used = torch.clamp(ratio, 0, 1 + config.epsilon)
        pol = lp * adv * r_used.detach()
    loss = -((pol - kl_c * kl + ent_c * ent) * w * mask).nan_to_num(0).sum()
    nl = batch.num_labels[:, 1:]
    stats = {"loss": float(loss), "ratio_new_old_sum": float((r_used * mask).sum()),
             "ratio_new_old_squared_sum": float((r_used * r_used * mask).sum()),
             "num_output_tokens_sum": int(mask.sum()), "entropy": float((ent / nl * mask).nan_to_num(0).sum())}
    return loss, stats
