"""Episode / Experience with the reference's fields and conversions
(src/environments/episode.py:5-84); Player mirrors src/backgammon/types/moves.py:36-42."""
from enum import IntEnum

import numpy as np
import torch


class Player(IntEnum):
    PLAYER1 = 0
    PLAYER2 = 1


class Experience:
    def __init__(self, observation, state_value, reward, done, next_observation, next_state_value):
        self.observation = observation
        self.state_value = state_value
        self.reward = reward
        self.done = done
        self.next_observation = next_observation
        self.next_state_value = next_state_value

    def to_numpy(self):
        for attr in vars(self):
            val = getattr(self, attr)
            if isinstance(val, torch.Tensor):
                setattr(self, attr, val.cpu().numpy())
            elif val is not None and hasattr(val, "to_numpy"):
                val.to_numpy()

    def to_tensor(self, device=None):
        # same type dispatch order as the reference (episode.py:30-46): a bool
        # matches `int` first and becomes an int64 tensor
        for attr in vars(self):
            val = getattr(self, attr)
            if isinstance(val, np.ndarray):
                setattr(self, attr, torch.from_numpy(val).to(device))
            elif isinstance(val, float):
                setattr(self, attr, torch.tensor(val, dtype=torch.float32, device=device))
            elif isinstance(val, int):
                setattr(self, attr, torch.tensor(val, dtype=torch.int64, device=device))
            elif isinstance(val, bool):
                setattr(self, attr, torch.tensor(val, dtype=torch.bool, device=device))
            elif isinstance(val, torch.Tensor) and device is not None:
                setattr(self, attr, val.to(device))
            elif val is not None and hasattr(val, "to_tensor"):
                val.to_tensor(device=device)


class Episode:
    def __init__(self):
        self.experiences = []
        self.win_type = None
        self.close_out_counts = {}
        self.prime_reward_counts = {}

    def add_experience(self, experience, info):
        self.experiences.append(experience)
        if info.get("win_type"):
            self.win_type = info["win_type"]
        current_player = info.get("current_player", None)
        if current_player is not None:
            if current_player not in self.close_out_counts:
                self.close_out_counts[current_player] = 0
            if current_player not in self.prime_reward_counts:
                self.prime_reward_counts[current_player] = 0
            if info.get("close_out_reward", False):
                self.close_out_counts[current_player] += 1
            if info.get("prime_reward", False):
                self.prime_reward_counts[current_player] += 1

    def to_numpy(self):
        for experience in self.experiences:
            experience.to_numpy()

    def to_tensor(self, device=None):
        for experience in self.experiences:
            experience.to_tensor(device=device)
