"""Test-fixture base model: restatement of the reference's ``CompatibleGCN``
(``src/gnn/model.py:7-53``): two dense propagations ``adj/deg @ x`` with
Linear layers.  Used only to exercise the WATS drop-in (it is the base model
the reference harness wraps, ``benchmark_calibration_methods.py:178-179``)."""
import torch
import torch.nn.functional as F
from torch import nn


class CompatibleGCN(nn.Module):
    def __init__(self, nfeat, nclass, nhid=64, dropout=0.5):
        super().__init__()
        self.gc1 = nn.Linear(nfeat, nhid)
        self.gc2 = nn.Linear(nhid, nclass)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x, adj):
        device = next(self.parameters()).device
        x = x.to(device)
        adj = adj.to(device)
        deg = adj.sum(dim=1, keepdim=True)
        deg[deg == 0] = 1
        adj_norm = adj / deg
        x = torch.mm(adj_norm, x)
        x = F.relu(self.gc1(x))
        x = self.dropout(x)
        x = torch.mm(adj_norm, x)
        return self.gc2(x)
