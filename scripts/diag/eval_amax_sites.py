"""Which evaluation tensors still take a standalone max-|x| pass (amax_kernel) and which
launches allocate zeroed memory, per evaluation chunk (GPU diagnostic)."""
import collections
import traceback

import torch

from dba_mod_amd import config as C
from dba_mod_amd.fl.plan import build_round_plan, select_clients
from dba_mod_amd.fl.server import Server
from dba_mod_amd.ops import hip as H
from dba_mod_amd.parallel.dist import DistCtx

sites = collections.Counter()
orig = H._amax


def spy(*a, **k):
    st = [f for f in traceback.extract_stack()[:-1] if "dba_mod_amd" in f.filename]
    sites[" <- ".join(f"{f.name}:{f.lineno}" for f in st[-4:])] += 1
    return orig(*a, **k)


H._amax = spy
zs = collections.Counter()
oz = torch.zeros


def zspy(*a, **k):
    st = [f for f in traceback.extract_stack()[:-1] if "dba_mod_amd" in f.filename]
    if st:
        zs[" <- ".join(f"{f.name}:{f.lineno}" for f in st[-3:])] += 1
    return oz(*a, **k)


p = C.load_params("configs/cifar_params.yaml", {"resumed_model": False, "synthetic_data": True,
                                                "start_epoch": 203, "overlap_eval": False})
s = Server(p, DistCtx(device=torch.device("cuda")), write_outputs=False)
agents, adv = select_clients(p, s.wl, 203)
plan = build_round_plan(p, s.wl, 203, agents, adv)
bank = s.global_state[None].repeat(3, 1)
jobs = plan.jobs[:3]
torch.zeros = zspy
s.evaluator.run(bank, [j.__class__(**{**j.__dict__, "model": i}) for i, j in enumerate(jobs)], 0, 1, None)
torch.zeros = oz
torch.cuda.synchronize()
print("amax sites:")
for k, v in sites.most_common():
    print(v, k)
print("zeros sites:")
for k, v in zs.most_common():
    print(v, k)
