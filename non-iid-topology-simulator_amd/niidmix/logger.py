"""Consensus distance on the GPU: the same "consensus-distance" event as
Logger.log_consensus_distance (tools/simulate/logger.py:257-284), computed by k_mean_cols +
k_row_dist2 over the [N, P] slab instead of N model_distance() calls on CPU models.

  event = consensus_distance_event(state)       # dict, reference schema (doc/experiment.md)
  log_consensus_distance(logger, state)         # appends it to logger.global_events
  install(Logger)                               # Logger.log_consensus_distance = GPU version

The uniform average is bit-identical to setup.model.average(models) (exact kernel); distances are
accumulated in fp64 (the reference accumulates fp32 per tensor), so they agree to ~1e-6 relative.
"""
import json
import statistics
import time

from .model import consensus_distance


def consensus_distance_event(state):
    models = [n["model"] for n in state["nodes"]]
    _, distances, norm = consensus_distance(models)
    return {
        "type": "consensus-distance",
        "step": state["step"],
        "distance_to_center": {
            "global": {
                "avg": statistics.mean(distances),
                "std": statistics.stdev(distances) if len(distances) > 1 else 0.,
                "max": max(distances),
                "min": min(distances),
            }
        },
        "center": {"norm": norm},
        "timestamp": time.strftime("%Y-%m-%d-%H:%M:%S-%Z"),
    }


def log_consensus_distance(logger, state):
    with open(logger.global_events, "a") as events:
        events.write(json.dumps(consensus_distance_event(state)) + "\n")


def install(logger_class):
    """Route a reference Logger class's log_consensus_distance through the GPU."""
    logger_class.log_consensus_distance = log_consensus_distance
    return logger_class

