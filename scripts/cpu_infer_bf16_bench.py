import sys, time
sys.path.insert(0, "/root/repo")
import torch
torch.set_num_threads(1)
from ray_amd.rllib.core.rl_module import RLModule
from ray_amd.rllib.env import make_env
env = make_env("SyntheticAtari-v0")
x = torch.randint(0, 256, (5, 84, 84, 4), dtype=torch.uint8)
def bench(f, n=100):
    for _ in range(10): f()
    t0 = time.perf_counter()
    for _ in range(n): f()
    return (time.perf_counter() - t0) / n * 1e3
m = RLModule(env.observation_space, env.action_space, {"vf_share_layers": True}).eval().to(memory_format=torch.channels_last)
with torch.no_grad():
    def ac():
        with torch.autocast("cpu", dtype=torch.bfloat16):
            return m.forward_inference(x)
    print("autocast bf16:", bench(ac))
    print("fp32:", bench(lambda: m.forward_inference(x)))
    mb = RLModule(env.observation_space, env.action_space, {"vf_share_layers": True}).eval().to(torch.bfloat16).to(memory_format=torch.channels_last)
    xb = x
    def pure():
        xx = xb.to(torch.bfloat16).mul_(1/255.)
        return mb.encoder.convs(xx.permute(0,3,1,2)) if hasattr(mb, "encoder") else None
    enc = [mm for mm in mb.modules() if hasattr(mm, "convs")][0]
    def pure2():
        xx = x.to(torch.bfloat16).mul_(1/255.).permute(0,3,1,2)
        h = enc.convs(xx)
        return enc.fc(h.permute(0,2,3,1).flatten(1))
    print("pure bf16 encoder:", bench(pure2))
    def ac_enc():
        with torch.autocast("cpu", dtype=torch.bfloat16):
            xx = x.float().mul_(1/255.).permute(0,3,1,2)
            h = [mm for mm in m.modules() if hasattr(mm, "convs")][0].convs(xx)
            return h
    print("autocast encoder convs only:", bench(ac_enc))
    # full pure-bf16 forward: weights bf16, uint8 frames cast straight to bf16
    pi = [mm for n, mm in mb.named_modules() if n in ("pi", "policy_head", "pi_head")]
    def pure_full():
        xx = x.to(torch.bfloat16).mul_(1/255.).permute(0,3,1,2)
        h = enc.fc(enc.convs(xx).permute(0,2,3,1).flatten(1))
        return [p(h) for p in pi]
    print("pure bf16 full (encoder+pi):", bench(pure_full), [n for n, _ in mb.named_children()])
    for th in (2,):
        torch.set_num_threads(th)
        print(f"threads={th} fp32:", bench(lambda: m.forward_inference(x)), "autocast:", bench(ac), "pure bf16 enc:", bench(pure2))
