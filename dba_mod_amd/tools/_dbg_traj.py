import sys, os, logging
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from dba_mod_amd import config as C
from dba_mod_amd.fl.server import Server
from dba_mod_amd.parallel.dist import init_distributed
dctx = init_distributed(prefer_gpu=True)
root = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
for method in sys.argv[1:]:
    p = C.load_params(f'{root}/configs/cifar_params.yaml', {"resumed_model": False, "synthetic_data": True,
         "save_dir": "/tmp/dbg", "aggregation_methods": method, "start_epoch": 100})
    s = Server(p, dctx, write_outputs=False)
    logging.getLogger("logger").setLevel(logging.WARNING)
    for e in range(100, 108):
        r = s.run_round(e)
        st = s.global_state
        v = s.spec.view(st[None], "bn1.running_var")
        print(method, e, round(r["global_acc"], 2), "rv min/max", float(v.min()) if v is not None else None,
              float(v.max()) if v is not None else None, "norm", float(st.double().norm()), flush=True)
