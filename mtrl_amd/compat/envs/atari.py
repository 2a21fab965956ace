"""AtariConfig (mtrl/envs/atari.py): the spaces the DrQ path is built from.  ALE stepping is host
env work, out of scope here; spawning the vector env needs gymnasium + ale-py,
which this image lacks, and raises."""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .spaces import Box, Discrete


@dataclass(frozen=True)
class AtariConfig:
    env_id: str = "atari-26"
    frame_stack: int = 4
    image_size: int = 84
    num_actions: int = 18  # the full ALE action set (drqeps.py:75 hardcodes 18)

    @property
    def observation_space(self):
        return Box(0, 255, (self.frame_stack, self.image_size, self.image_size), np.uint8)

    @property
    def action_space(self):
        return Discrete(self.num_actions)

    def spawn(self, *args, **kwargs):
        raise NotImplementedError("Atari environments (gymnasium + ale-py) are not installed in this image")
