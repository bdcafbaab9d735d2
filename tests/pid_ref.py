"""Numpy restatement of ballbot_gym/controllers/pid.py:PID.act (test helper).

Used as a closed-loop behavioural check (scripts/test_pid.py:32-63 balances
the robot on flat terrain with gains 20/15/2)."""
import numpy as np


class PID:
    def __init__(self, dt, k_p, k_i, k_d):
        self.k_p, self.k_i, self.k_d, self.dt = k_p, k_i, k_d, dt
        self.integral = np.zeros(2, np.float32)
        self.prev_err = np.zeros(2, np.float32)

    def act(self, R):  # pid.py:49-101 (return in motor space)
        R = np.asarray(R, np.float32)
        roll = np.arctan2(R[2, 1], R[2, 2])
        pitch = np.arctan2(-R[2, 0], np.sqrt(R[2, 1] ** 2 + R[2, 2] ** 2))
        err = np.array([0 - pitch, 0 - roll], np.float32)
        self.integral += err * self.dt
        deriv = (err - self.prev_err) / self.dt
        u = self.k_p * err + self.k_i * self.integral + self.k_d * deriv
        self.prev_err = err
        c = np.zeros(3, np.float32)
        for k, a in enumerate((0, 120, 240)):
            c[k] = u[1] * np.cos(np.deg2rad(a)) + u[0] * np.sin(np.deg2rad(a))
        return np.clip(c, -10, 10)


def rotvec_to_R(rv):
    rv = np.asarray(rv, np.float64)
    th = np.linalg.norm(rv)
    if th < 1e-14:
        return np.eye(3)
    k = rv / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
