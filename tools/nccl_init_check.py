import os, torch, torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29555")
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
dist.barrier(); t = torch.ones(4, device=dev); dist.all_reduce(t); torch.cuda.synchronize()
print("nccl device_id ok", t.tolist()); dist.destroy_process_group()
