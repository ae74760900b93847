"""MEASUREMENT TOOL (not the product path): the reference's rl_step loss head as the same
ATen op chain (pipelinerl/finetune/rl/__init__.py:199-292 + rl/utils.py sum_sum with its
per-segment Python loop), runnable on the GPU, so the fused HIP kernel can be timed against
the reference's own approach on the same MI355X.  Returns (loss, minimal stats); backward
through autograd as in the reference.
"""

import torch
import torch.nn.functional as F


def _sum_sum(values, masks, segments):
    if segments and values.shape[-1] != 1:
        return torch.stack([(values[0, a:b] * masks[0, a:b]).nan_to_num(0).sum() for a, b in segments]).sum()
    return (values * masks).nan_to_num(0).sum()


def aten_loss_head(logits, batch, config, current_step=0, max_step=100):
    masks = batch.labels != -100
    masks_shifted = masks[:, 1:]
    pos = batch.position_ids[0]
    starts = pos == 0
    starts[0] = True
    seq_starts = torch.where(starts)[0]
    bounds = torch.cat([seq_starts, torch.tensor([pos.shape[0]], device=pos.device)])
    segments = list(zip(bounds[:-1], bounds[1:]))
    x = logits[:, :-1, :] / config.temperature
    logprobs = F.log_softmax(x, dim=-1)
    probs = F.softmax(x, dim=-1)
    entropy = -(probs * logprobs).sum(dim=-1)
    new_lp = torch.gather(logprobs, 2, batch.input_ids[:, 1:].unsqueeze(2)).squeeze(2)
    assert torch.isfinite(new_lp).all()
    ref = batch.ref_logprobs[:, 1:]
    old = batch.old_logprobs[:, 1:]
    w = torch.ones_like(batch.group_tokens[:, 1:]) / config.batch_size
    ratio = torch.exp(new_lp - old)
    lrrn = ref - new_lp
    assert torch.isfinite(lrrn).all()
    adv = batch.advantages[:, 1:]
    C = config.clamp_log_ratio_ref_new_value
    c = torch.clamp(lrrn, -C, C)
    kl = torch.exp(c) - c - 1
    assert torch.isfinite(kl).all()
    frac = current_step / max_step
    kl_c = config.kl_coef + (config.final_kl_coef - config.kl_coef) * frac
    ent_c = config.entropy_bonus + (config.final_entropy_bonus - config.entropy_bonus) * frac
    surr1 = ratio * adv
    surr2 = torch.clamp(ratio, 1 - config.epsilon, 1 + config.epsilon) * adv
    pol = torch.min(surr1, surr2)
    loss = (pol - kl_c * kl + ent_c * entropy) * w
    final = -_sum_sum(loss, masks_shifted, segments)
    assert torch.isfinite(final)
    nl = batch.num_labels[:, 1:]
    stats = {"loss": final.item(), "entropy": _sum_sum(entropy / nl, masks_shifted, segments).item(),
             "kl": _sum_sum(kl / nl, masks_shifted, segments).item(),
             "ratio_new_old_sum": _sum_sum(ratio, masks_shifted, segments).item()}
    return final, stats
