"""Tracker registry — drop-in for boxmot.tracker_zoo (reference boxmot/tracker_zoo.py:8-93).

Same names, same argument meaning, same YAML-default extraction and the same error behaviour
for unknown names (prints, then KeyError).  Registered trackers whose association path is not on
the MI355X engine yet raise NotImplementedError.
"""
from __future__ import annotations

from pathlib import Path

import yaml

TRACKER_CONFIGS = Path(__file__).resolve().parent / "configs" / "trackers"

_ON_ENGINE = {
    "bytetrack": "boxmot_amd.trackers.bytetrack.ByteTrack",
    "botsort": "boxmot_amd.trackers.botsort.BotSort",
    "ocsort": "boxmot_amd.trackers.ocsort.OcSort",
    "boosttrack": "boxmot_amd.trackers.boosttrack.BoostTrack",
    "strongsort": "boxmot_amd.trackers.strongsort.StrongSort",
}
_REFERENCE_NAMES = ["strongsort", "ocsort", "bytetrack", "botsort", "deepocsort", "hybridsort",
                    "boosttrack"]


def get_tracker_config(tracker_type):
    """Path to the tracker's YAML configuration (tracker_zoo.py:8-10)."""
    return TRACKER_CONFIGS / f"{tracker_type}.yaml"


def create_tracker(tracker_type, tracker_config=None, reid_weights=None, device=None, half=None,
                   per_class=None, evolve_param_dict=None):
    if evolve_param_dict is None:
        cfg = tracker_config if tracker_config is not None else get_tracker_config(tracker_type)
        with open(cfg, "r") as f:
            yaml_config = yaml.safe_load(f)
        tracker_args = {param: details["default"] for param, details in yaml_config.items()}
    else:
        tracker_args = dict(evolve_param_dict)
    reid_args = {"reid_weights": reid_weights, "device": device, "half": half}
    if tracker_type not in _REFERENCE_NAMES:
        print("Error: No such tracker found.")
        raise KeyError(tracker_type)
    if tracker_type not in _ON_ENGINE:
        raise NotImplementedError(f"{tracker_type} is not on the MI355X association engine yet")
    module_path, class_name = _ON_ENGINE[tracker_type].rsplit(".", 1)
    cls = getattr(__import__(module_path, fromlist=[class_name]), class_name)
    if tracker_type in ["strongsort", "botsort", "deepocsort", "hybridsort", "boosttrack"]:
        tracker_args["per_class"] = per_class
        tracker_args.update(reid_args)
        if tracker_type in ["strongsort"]:
            tracker_args.pop("per_class")  # tracker_zoo.py:84-85
    else:
        tracker_args["per_class"] = per_class
    return cls(**tracker_args)
