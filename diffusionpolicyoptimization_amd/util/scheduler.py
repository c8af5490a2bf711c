"""LR schedules (reference util/scheduler.py). Host scalars: evaluated once per optimiser step."""
import math


class CosineAnnealingWarmupRestarts2:
    """util/scheduler.py:67-177 semantics: warm up from initial_learning_rate to max_lr, then cosine
    back to initial_learning_rate; called with the optimiser's iteration count (Keras calls the
    schedule with `iterations`). At the shipped cfgs (initial = max) the rate is constant."""

    def __init__(self, initial_learning_rate, first_cycle_steps, cycle_mult=1.0, max_lr=0.1, min_lr=0.001,
                 warmup_steps=0, gamma=1.0, last_epoch=-1):
        assert warmup_steps < first_cycle_steps
        self.initial_learning_rate = initial_learning_rate
        self.first_cycle_steps = first_cycle_steps
        self.cycle_mult = cycle_mult
        self.base_max_lr = max_lr
        self.max_lr = max_lr
        self.min_lr = min_lr
        self.warmup_steps = warmup_steps
        self.gamma = gamma
        self.cur_cycle_steps = first_cycle_steps
        self.cycle = 0
        self.step_in_cycle = last_epoch

    def get_lr(self):
        if self.step_in_cycle == -1:
            return self.initial_learning_rate
        if self.step_in_cycle < self.warmup_steps:
            return (self.max_lr - self.initial_learning_rate) * self.step_in_cycle / self.warmup_steps \
                + self.initial_learning_rate
        frac = (int(self.step_in_cycle) - self.warmup_steps) / (self.cur_cycle_steps - self.warmup_steps)
        return self.initial_learning_rate + (self.max_lr - self.initial_learning_rate) * \
            (1 + math.cos(math.pi * frac)) / 2

    def __call__(self, step):
        step = int(step)
        if step >= self.first_cycle_steps:
            if self.cycle_mult == 1.0:
                self.step_in_cycle = step % self.first_cycle_steps
                self.cycle = step // self.first_cycle_steps
            else:
                n = int(math.log(step / self.first_cycle_steps * (self.cycle_mult - 1) + 1, self.cycle_mult))
                self.cycle = n
                self.step_in_cycle = step - int(self.first_cycle_steps * (self.cycle_mult ** n - 1) /
                                                (self.cycle_mult - 1))
                self.cur_cycle_steps = self.first_cycle_steps * self.cycle_mult ** n
        else:
            self.cur_cycle_steps = self.first_cycle_steps
            self.step_in_cycle = step
        self.max_lr = self.base_max_lr * (self.gamma ** self.cycle)
        self.last_epoch = math.floor(step)
        return self.get_lr()


class CosineAnnealingWarmupRestarts:
    """util/scheduler.py:6-64 (used for eta only): min_lr -> max_lr warmup, cosine back to min_lr."""

    def __init__(self, first_cycle_steps, cycle_mult=1.0, max_lr=0.1, min_lr=0.001, warmup_steps=0, gamma=1.0):
        assert warmup_steps < first_cycle_steps
        self.first_cycle_steps, self.cycle_mult = first_cycle_steps, cycle_mult
        self.max_lr, self.min_lr, self.warmup_steps, self.gamma = max_lr, min_lr, warmup_steps, gamma

    def __call__(self, step):
        start, cyc, n = 0, self.first_cycle_steps, 0
        while step >= start + cyc:
            start += cyc
            cyc = int((cyc - self.warmup_steps) * self.cycle_mult + self.warmup_steps)
            n += 1
        s = step - start
        max_lr = self.max_lr * (self.gamma ** n)
        if s < self.warmup_steps:
            return self.min_lr + (max_lr - self.min_lr) * s / self.warmup_steps
        prog = (s - self.warmup_steps) / (cyc - self.warmup_steps)
        return self.min_lr + (max_lr - self.min_lr) * (1 + math.cos(math.pi * prog)) / 2


class CosineDecayRestarts:
    """tf.keras.optimizers.schedules.CosineDecayRestarts as the pretrain agent builds it
    (agent/pretrain/train_agent.py:117-123): lr(step) = initial * ((1 - alpha) * m_mul^i *
    (1 + cos(pi * frac)) / 2 + alpha), with the restart index i and in-cycle fraction frac of
    step / first_decay_steps under t_mul."""

    def __init__(self, initial_learning_rate, first_decay_steps, t_mul=2.0, m_mul=1.0, alpha=0.0):
        self.initial_learning_rate = float(initial_learning_rate)
        self.first_decay_steps = float(first_decay_steps)
        self.t_mul, self.m_mul, self.alpha = float(t_mul), float(m_mul), float(alpha)

    def __call__(self, step):
        frac = float(step) / self.first_decay_steps
        if self.t_mul == 1.0:
            i = math.floor(frac)
            frac -= i
        else:
            i = math.floor(math.log(1.0 - frac * (1.0 - self.t_mul)) / math.log(self.t_mul))
            sum_r = (1.0 - self.t_mul ** i) / (1.0 - self.t_mul)
            frac = (frac - sum_r) / self.t_mul ** i
        cos_decay = 0.5 * self.m_mul ** i * (1.0 + math.cos(math.pi * frac))
        return self.initial_learning_rate * ((1.0 - self.alpha) * cos_decay + self.alpha)
