"""Diagnose run-to-run gradient differences: two processes computing the same
slice's gradients concurrently on one GPU vs one process alone."""
import os, sys, socket
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import torch, torch.distributed as dist, torch.multiprocessing as mp
import test_gpu_dist as T

def err(a, b):
    den = float(torch.linalg.vector_norm(b.double()))
    return float(torch.linalg.vector_norm(a.double() - b.double())) / den if den > 0 else 0.0

def grads(model, recipe):
    model.zero_grad(set_to_none=True)
    T._loss(model, *T._slice(recipe, 0)).backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}

def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model, recipe = T._setup(rank)
    dist.barrier()
    conc = grads(model, recipe)              # both processes at once
    dist.barrier()
    if rank == 0:
        alone = [grads(model, recipe) for _ in range(2)]
        e1 = {n: err(conc[n], alone[0][n]) for n in conc}
        e0 = max(err(alone[1][n], alone[0][n]) for n in conc)
        top = sorted(e1, key=lambda n: -e1[n])[:4]
        print("alone vs alone:", e0, flush=True)
        print("concurrent vs alone:", [(n[-45:], "%.2e" % e1[n]) for n in top], flush=True)
    dist.barrier(); dist.destroy_process_group()

if __name__ == "__main__":
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]
    mp.spawn(worker, args=(2, port), nprocs=2, join=True)
