"""AdamW over the flat [actor_ft | critic] buffer on the device (dppo_adamw).

Default semantics are Keras 3 AdamW as the reference constructs it (train_ppo_agent.py:45-49):
`decay=` is not weight decay in Keras 3, so the default weight_decay = 0.004 applies to every
variable, decoupled and before the Adam step, epsilon = 1e-7, and ONE optimiser trains actor_ft
and critic at the actor LR (the critic optimiser is never applied, agent :360). mode="torch"
gives PyTorch AdamW as a documented alternative."""
from .. import ops


class AdamW:
    def __init__(self, params, learning_rate, weight_decay=0.004, beta_1=0.9, beta_2=0.999, epsilon=1e-7,
                 mode="keras"):
        import torch
        self.params = params
        self.m = torch.zeros_like(params)
        self.v = torch.zeros_like(params)
        self.learning_rate = learning_rate
        self.weight_decay, self.beta_1, self.beta_2, self.epsilon = weight_decay, beta_1, beta_2, epsilon
        self.mode = mode
        self.iterations = 0

    def current_lr(self):
        lr = self.learning_rate
        return float(lr(self.iterations)) if callable(lr) else float(lr)

    def apply_gradients(self, grads):
        lr = self.current_lr()
        self.iterations += 1
        ops.adamw(self.params, grads, self.m, self.v, self.iterations, lr, self.weight_decay, self.beta_1, self.beta_2,
                  self.epsilon, self.mode)
        return lr

    def begin_step(self):
        """Advance the step counter for one optimiser step applied in parts (apply_range)."""
        lr = self.current_lr()
        self.iterations += 1
        return lr

    def apply_range(self, grads, lo, hi, lr, dims=None, precision=None, packs=(), metrics=None, metrics_out=None,
                    n_metrics=0, metrics_tag=0, defer_sampler_tables=False):
        """The step begin_step() opened, over params[lo:hi], then the images in `packs`
        ((actor_params, packed_actor) and/or (critic_params, packed_critic), keyed "actor" /
        "critic") re-derived, with the minibatch's metric sums copied to metrics_out (followed by
        metrics_tag when nonzero): one dppo_optimizer_step call (two launches) on the current stream.
        defer_sampler_tables: the actor's split-sampler tables wait for the next sampler launch."""
        pk = dict(packs)
        ap, pa = pk.get("actor", (None, None))
        cp, pc = pk.get("critic", (None, None))
        ops.optimizer_step(dims, precision, self.params[lo:hi], grads[lo:hi], self.m[lo:hi], self.v[lo:hi],
                           self.iterations, lr, self.weight_decay, self.beta_1, self.beta_2, self.epsilon, self.mode,
                           ap, pa, cp, pc, metrics, metrics_out, n_metrics, metrics_tag,
                           defer_sampler_tables=defer_sampler_tables)

    def bind_range(self, grads, lo, hi, dims, precision, packs=(), defer_sampler_tables=False, l2_from_pl2=False,
                   fused_pack=False, clear_grads=False):
        """apply_range over a fixed range and fixed images, validated and marshalled once
        (ops.BoundOptimizerStep): returns f(lr, metrics=None, metrics_out=None, n_metrics=0,
        metrics_tag=0, stream=None, clear=None) for the step begin_step() opened. fused_pack /
        clear_grads: ABI 11 (one launch; the gradients and the `clear` ranges zeroed after use)."""
        pk = dict(packs)
        ap, pa = pk.get("actor", (None, None))
        cp, pc = pk.get("critic", (None, None))
        b = ops.BoundOptimizerStep(dims, precision, self.params[lo:hi], grads[lo:hi], self.m[lo:hi], self.v[lo:hi],
                                   self.weight_decay, self.beta_1, self.beta_2, self.epsilon, self.mode, ap, pa, cp,
                                   pc, defer_sampler_tables=defer_sampler_tables, l2_from_pl2=l2_from_pl2,
                                   fused_pack=fused_pack, clear_grads=clear_grads)

        def step(lr, metrics=None, metrics_out=None, n_metrics=0, metrics_tag=0, stream=None, clear=None):
            b(self.iterations, lr, metrics, metrics_out, n_metrics, metrics_tag, stream=stream, clear=clear)
        return step

    def apply_gradients_split(self, grads, ranges):
        """One optimiser step over disjoint ranges of the flat buffer, each on its own stream:
        ranges = [(lo, hi, stream), ...]. Elementwise, so it equals apply_gradients."""
        import torch
        lr = self.current_lr()
        self.iterations += 1
        for lo, hi, st in ranges:
            with torch.cuda.stream(st):
                ops.adamw(self.params[lo:hi], grads[lo:hi], self.m[lo:hi], self.v[lo:hi], self.iterations, lr,
                          self.weight_decay, self.beta_1, self.beta_2, self.epsilon, self.mode)
        return lr

    def state_dict(self):
        return {"m": self.m.detach().cpu().numpy(), "v": self.v.detach().cpu().numpy(), "iterations": self.iterations}

    def load_state_dict(self, d):
        import torch
        self.m.copy_(torch.as_tensor(d["m"]))
        self.v.copy_(torch.as_tensor(d["v"]))
        self.iterations = int(d["iterations"])
