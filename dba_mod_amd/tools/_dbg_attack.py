import sys, os, logging, csv
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from dba_mod_amd import config as C
from dba_mod_amd.fl.server import Server
from dba_mod_amd.parallel.dist import init_distributed
dctx = init_distributed(prefer_gpu=True)
root = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
cfg = sys.argv[1] if len(sys.argv) > 1 else "cifar_params"
p = C.load_params(f'{root}/configs/{cfg}.yaml', {"resumed_model": False, "synthetic_data": True,
     "save_dir": "/tmp/dbg", "start_epoch": 201, "pretrain_rounds": 20})
s = Server(p, dctx, write_outputs=True, folder="/tmp/dbg/run")
logging.getLogger("logger").setLevel(logging.WARNING)
for e in range(201, 211):
    r = s.run_round(e)
    print("round", e, round(r["global_acc"], 2), round(r["global_asr"], 2), flush=True)
for f in ("posiontest_result.csv", "poisontriggertest_result.csv", "scale_result.csv", "train_result.csv"):
    rows = list(csv.reader(open(os.path.join("/tmp/dbg/run", f))))
    print("==", f)
    for row in rows:
        if f == "train_result.csv" and not any(x in row[0] for x in ("17", "33", "77", "11")):
            continue
        print(row)
