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


class DistributedParameterManager:
    """The ParameterManager surface for one process per GPU.

    The reference shares weights through a Manager dict polled by every worker
    (parameter_manager.py:79-111, worker.py:66-76). Here the trainer rank
    (`src`) owns the weights: set_parameters() stores them and bumps the
    version locally; every rank calls sync() at its harvest cadence, which is
    one 8-byte version broadcast and, only when the version moved, the
    102,404-byte weight broadcast (bgx.dist.broadcast_weights, RCCL over xGMI
    with the nccl backend). A rank's Engine (optional) is re-armed with the new
    weights and the reference's temperature schedule on the spot.
    """

    INITIAL_TEMPERATURE = INITIAL_TEMPERATURE
    FINAL_TEMPERATURE = FINAL_TEMPERATURE
    MAX_UPDATES = MAX_UPDATES

    def __init__(self, engine=None, src=0, state_dict=None):
        import torch.distributed as dist

        self.dist = dist
        self.src = src
        self.engine = engine
        self.version = 0
        self._applied = 0      # version whose weights this rank holds / its engine runs
        self.weights = None
        if dist.get_rank() == src:
            sd = state_dict if state_dict is not None else BackgammonPolicyNetwork().state_dict()
            self.weights = _to_weights(sd)
            self.version = 1
        self.sync()

    def _device(self):
        if self.dist.get_backend() == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def set_parameters(self, new_state_dict):
        """Trainer rank only: takes effect everywhere at the next sync()."""
        if self.dist.get_rank() != self.src:
            raise RuntimeError("set_parameters is the trainer rank's call")
        self.weights = _to_weights(new_state_dict)
        self.version += 1

    def sync(self):
        """Collective (all ranks): propagate a version bump. Returns True if the
        weights changed on this rank."""
        from bgx.dist import broadcast_weights

        v = torch.tensor([self.version], dtype=torch.int64, device=self._device())
        self.dist.broadcast(v, src=self.src)
        v = int(v.item())
        if v == self._applied:
            return False
        self.weights = broadcast_weights(self.weights if self.weights is not None else {}, src=self.src)
        self.version = v
        self._applied = v
        if self.engine is not None:
            self.engine.set_weights(self.weights, self.get_temperature(), v)
        return True

    def get_parameters(self, device=None):
        names = {"W1": "fc1.weight", "b1": "fc1.bias", "w2": "value_head.weight", "b2": "value_head.bias"}
        shapes = {"W1": (128, 198), "b1": (128,), "w2": (1, 128), "b2": (1,)}
        return {names[k]: torch.as_tensor(self.weights[k].reshape(shapes[k]), device=device) for k in names}

    def get_version(self):
        return self.version

    def get_temperature(self):
        v = self.version
        if v <= 1:
            return self.INITIAL_TEMPERATURE
        if v >= 1 + self.MAX_UPDATES:
            return self.FINAL_TEMPERATURE
        frac = (v - 1) / self.MAX_UPDATES
        return self.INITIAL_TEMPERATURE - (self.INITIAL_TEMPERATURE - self.FINAL_TEMPERATURE) * frac


def _to_weights(sd):
    from bgx.ops import weights_from
    return dict(zip(("W1", "b1", "w2", "b2"), weights_from(sd)))
