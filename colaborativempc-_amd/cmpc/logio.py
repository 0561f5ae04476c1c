"""Experiment log / wire formats of the reference, so its MATLAB post-processing
("planner/matlab scripts/mainComp.m", tools/import_*.m) reads our runs unchanged.

* ``save_to_csv``: <path_csv>/csv/<id>/{states,u,plan_dist,time}.dat (+ time_OCD.dat,
  OCD_it.dat for OCD runs) as ``np.savetxt(fmt='%.5e', delimiter=' ')``
  (plan_lib/config/base_class.py:64-99, with time / time_OCD of :143-166).
* ``save_settings``: settings.csv, one ``key,value`` row per config entry (utilities/misc.py:264-275).
* ``serialise_np`` / ``deserialise_np``: the ROS ``agent_info`` payload (a list of float32
  arrays with their shapes; ROS/src/planner_experiments/src/utilities_ROS/utilities_ros.py:7-45),
  for interop with the reference's ROS nodes.
"""
from __future__ import annotations

import csv
import os

import numpy as np

FMT = "%.5e"


def _time_agg(time_op, ocd_it):
    """base_class.time (:156-166): per-step sum of the OCD round times."""
    if all(it == 0 for it in ocd_it):
        return np.asarray(time_op)
    out = np.zeros(len(ocd_it))
    for i, it in enumerate(ocd_it):
        out[i] = sum(time_op[i * it:(i + 1) * it])
    return out


def _time_ocd(time_op, ocd_it):
    """base_class.time_OCD (:143-154): per-step rows of the round times, zero padded."""
    if all(it == 0 for it in ocd_it):
        return np.asarray(time_op)
    lim = int(np.max(np.asarray(ocd_it)))
    out = np.zeros((len(ocd_it), lim))
    for i, it in enumerate(ocd_it):
        out[i, :it] = time_op[i * it:(i + 1) * it]
    return out


def save_to_csv(path_csv, agent_id, states, u, look_ahead, time_op, ocd_it=None):
    """states: first predicted state per step (rows), u: first input per step, look_ahead:
    xPred[-1, 6] - xPred[0, 6] per step, time_op: solve times (s)."""
    path = os.path.join(path_csv, "csv", str(agent_id))
    os.makedirs(path, exist_ok=True)
    np.savetxt(os.path.join(path, "states.dat"), np.asarray(states), fmt=FMT, delimiter=" ")
    np.savetxt(os.path.join(path, "u.dat"), np.asarray(u), fmt=FMT, delimiter=" ")
    np.savetxt(os.path.join(path, "plan_dist.dat"), np.asarray(look_ahead), fmt=FMT, delimiter=" ")
    if ocd_it is not None:
        np.savetxt(os.path.join(path, "time.dat"), _time_agg(time_op, ocd_it), fmt=FMT, delimiter=" ")
        np.savetxt(os.path.join(path, "time_OCD.dat"), _time_ocd(time_op, ocd_it), fmt=FMT, delimiter=" ")
        np.savetxt(os.path.join(path, "OCD_it.dat"), np.asarray(ocd_it), fmt=FMT, delimiter=" ")
    else:
        np.savetxt(os.path.join(path, "time.dat"), np.asarray(time_op), fmt=FMT, delimiter=" ")
    return path


def save_settings(path, settings):
    """settings.csv as utilities/misc.py:264-275 writes it (csv rows key,value)."""
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "settings.csv"), "w", newline="") as f:
        w = csv.writer(f)
        for k, v in settings.items():
            w.writerow([k, v])


def serialise_np(arrays):
    """List of arrays -> list of (float32 flat data, shape) as the ROS agent_info message
    carries them (Float32MultiArray with one dim per axis; utilities_ros.py:7-34)."""
    out = []
    for a in arrays:
        a = np.asarray(a, dtype=np.float32)
        out.append((a.ravel().copy(), tuple(a.shape)))
    return out


def deserialise_np(msgs):
    """Inverse of serialise_np (utilities_ros.py:36-45): float32 arrays back to their shapes."""
    return [np.asarray(d, dtype=np.float32).reshape(shape) for d, shape in msgs]
