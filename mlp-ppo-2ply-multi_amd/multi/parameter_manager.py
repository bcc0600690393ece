"""ParameterManager (src/multi/parameter_manager.py:17-230): versioned shared
weights + the linear temperature schedule. Same constructor (Manager lock,
Value, dict), same methods and numerics; S3 save/load is out of scope and
falls back to the local path with a warning."""
import os
import warnings

import torch

from bgx.net import BackgammonPolicyNetwork

INITIAL_TEMPERATURE = 1.5   # config/configuration.py:20-22
FINAL_TEMPERATURE = 0.5
MAX_UPDATES = 4000


class ParameterManager:
    INITIAL_TEMPERATURE = INITIAL_TEMPERATURE
    FINAL_TEMPERATURE = FINAL_TEMPERATURE
    MAX_UPDATES = MAX_UPDATES

    def __init__(self, lock, version, parameters):
        self.lock = lock
        self.version = version
        self.parameters = parameters
        with self.lock:
            if not bool(self.parameters):
                state_dict = {k: v.cpu() for k, v in BackgammonPolicyNetwork().state_dict().items()}
                self.parameters.update(state_dict)
                self.version.value = 1

    def get_parameters(self, device=None):
        return {key: torch.as_tensor(array, device=device) for key, array in self.parameters.items()}

    def get_version(self):
        return self.version.value

    def set_parameters(self, new_state_dict):
        with self.lock:
            for key, tensor in new_state_dict.items():
                self.parameters[key] = tensor.cpu().numpy()
            self.version.value += 1

    def get_temperature(self):
        v = self.get_version()
        if v <= 1:
            return self.INITIAL_TEMPERATURE
        if v >= 1 + self.MAX_UPDATES:
            return self.FINAL_TEMPERATURE
        frac = (v - 1) / self.MAX_UPDATES
        return self.INITIAL_TEMPERATURE - (self.INITIAL_TEMPERATURE - self.FINAL_TEMPERATURE) * frac

    def save_model_local(self, filename=None):
        os.makedirs("models", exist_ok=True)
        path = os.path.join("models", filename or "ppo_backgammon.pth")
        torch.save(self.get_parameters(), path)
        print(f"Model saved locally to {path}")

    def load_model_local(self, filename=None):
        path = os.path.join("models", filename or "ppo_backgammon.pth")
        if os.path.isfile(path):
            self.set_parameters(torch.load(path, map_location="cpu", weights_only=True))
            print(f"Model loaded locally from {path}")
        else:
            print(f"No saved model found locally at {path}")

    def save_model(self, filename=None, to_s3=False):
        if to_s3:
            warnings.warn("S3 upload is out of scope for the MI355X build; saving locally")
        self.save_model_local(filename)

    def load_model(self, filename=None, from_s3=False):
        if from_s3:
            warnings.warn("S3 download is out of scope for the MI355X build; loading locally")
        self.load_model_local(filename)
