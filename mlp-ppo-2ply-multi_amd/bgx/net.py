"""BackgammonPolicyNetwork (src/agents/policy_network.py:36-70) as a torch module.

Host-side plumbing only: it gives ParameterManager a state_dict with the
reference's keys/shapes (fc1.weight [128,198], fc1.bias, value_head.weight
[1,128], value_head.bias) and xavier-uniform init. Self-play evaluates the
network in libbgx.so (bgx_mlp.hip), never through this module.
"""
import torch
import torch.nn as nn


class BackgammonPolicyNetwork(nn.Module):
    def __init__(self, input_size=198, hidden_size=128):
        super().__init__()
        self.fc1 = nn.Linear(input_size, hidden_size)
        self.value_head = nn.Linear(hidden_size, 1)
        nn.init.xavier_uniform_(self.fc1.weight)
        nn.init.xavier_uniform_(self.value_head.weight)

    def forward(self, x):
        return self.value_head(torch.sigmoid(self.fc1(x))).squeeze(-1)
