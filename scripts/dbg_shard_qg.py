"""Debug: ShardedIndex QG search on a one-rank nccl group (test_gpu_shard)."""
import os, socket, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import torch
import torch.distributed as dist
from ngt_amd.shard import ShardedIndex
from ngt_amd.device import SEED_TREE
from test_gpu_qg import device_qg, state
s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(port)
dev = torch.device("cuda:0")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
_, _, _, _, _, _, _, z, meta, dim, _ = state("c1_qg")
qix = device_qg("c1_qg")
qsq = z["queries"].astype(np.float32)
d_q = torch.from_numpy(qsq).to(dev)
sq = ShardedIndex(torch, dist, qix, 0, dev)
stream = torch.cuda.current_stream(dev).cuda_stream
print("stream", stream, "dim", dim, "nq", len(qsq), flush=True)
key = "10_0.05_3"
k, eps, exp = key.split("_")
# the local search alone
ids, ds, n = sq._out(len(qsq), int(k))
qix.qg_search_device(d_q.data_ptr(), dim * 4, len(qsq), ids.data_ptr(), ds.data_ptr(), n.data_ptr(), None,
                     k=int(k), epsilon=float(eps), result_expansion=float(exp), seed_mode=SEED_TREE, stream=stream,
                     visited_hash_log2=-1)
torch.cuda.synchronize()
print("local n", n[:8].tolist(), "ids", ids[0].tolist(), flush=True)
gi, gd, gn = sq.merge_local(ids, ds, n, int(k), stream)
torch.cuda.synchronize()
print("merged n", gn[:8].tolist(), gi[0].tolist(), flush=True)
gi, gd, gn = sq.qg_search_device(d_q.data_ptr(), dim * 4, len(qsq), int(k), float(eps), result_expansion=float(exp),
                                 stream=stream, seed_mode=SEED_TREE)
torch.cuda.synchronize()
print("qg_search_device n", gn[:8].tolist(), gi[0].tolist(), flush=True)
print("ref", z["n_" + key][:8].tolist(), z["ids_" + key][0].tolist(), flush=True)
dist.destroy_process_group()
