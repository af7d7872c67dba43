"""Value schedules (reference: rllib/utils/schedules/): ``value(t)`` of a timestep."""

from __future__ import annotations


class Schedule:
    def __init__(self, framework=None):
        self.framework = framework

    def value(self, t):
        return self._value(t)

    def __call__(self, t):
        return self.value(t)

    def _value(self, t):
        raise NotImplementedError


class ConstantSchedule(Schedule):
    def __init__(self, value, framework=None):
        super().__init__(framework)
        self._v = value

    def _value(self, t):
        return self._v


class PolynomialSchedule(Schedule):
    """``final + (initial - final) * (1 - t / schedule_timesteps) ** power``, held at
    ``final_p`` after ``schedule_timesteps``."""

    def __init__(self, schedule_timesteps, final_p, framework=None, initial_p=1.0,
                 power=2.0):
        super().__init__(framework)
        self.schedule_timesteps = max(1, int(schedule_timesteps))
        self.final_p, self.initial_p, self.power = final_p, initial_p, power

    def _value(self, t):
        frac = min(float(t), self.schedule_timesteps) / self.schedule_timesteps
        return self.final_p + (self.initial_p - self.final_p) * (1.0 - frac) ** self.power


class LinearSchedule(PolynomialSchedule):
    def __init__(self, schedule_timesteps, final_p, framework=None, initial_p=1.0):
        super().__init__(schedule_timesteps, final_p, framework, initial_p, power=1.0)


class ExponentialSchedule(Schedule):
    """``initial_p * decay_rate ** (t / schedule_timesteps)``."""

    def __init__(self, schedule_timesteps, framework=None, initial_p=1.0, decay_rate=0.1):
        super().__init__(framework)
        self.schedule_timesteps = max(1, int(schedule_timesteps))
        self.initial_p, self.decay_rate = initial_p, decay_rate

    def _value(self, t):
        return self.initial_p * self.decay_rate ** (float(t) / self.schedule_timesteps)


class PiecewiseSchedule(Schedule):
    """Linear interpolation between ``endpoints`` [(t, value), ...]; ``outside_value``
    past the last one (the last value when None)."""

    def __init__(self, endpoints, framework=None, interpolation=None, outside_value=None):
        super().__init__(framework)
        self.endpoints = sorted((int(t), v) for t, v in endpoints)
        self.interpolation = interpolation or (lambda a, b, alpha: a + alpha * (b - a))
        self.outside_value = outside_value

    def _value(self, t):
        for (l_t, l_v), (r_t, r_v) in zip(self.endpoints[:-1], self.endpoints[1:]):
            if l_t <= t < r_t:
                return self.interpolation(l_v, r_v, float(t - l_t) / float(r_t - l_t))
        if t < self.endpoints[0][0]:
            return self.endpoints[0][1]
        return self.outside_value if self.outside_value is not None else self.endpoints[-1][1]


__all__ = ["Schedule", "ConstantSchedule", "LinearSchedule", "PiecewiseSchedule",
           "PolynomialSchedule", "ExponentialSchedule"]
