import sys, torch, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tools')
from channelestimationtransformer_amd.informer import InformerStack
from channelestimationtransformer_amd.weights import synthetic_state_dict
dev = torch.device("cuda:0")
m = InformerStack(16, 16, 16, 32, 10, 5, 5, 64, 4, [2, 1], 2, 64, 0.05, "full", "fixed", "gelu", False, True, dev)
m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(m._schema(), 3).items()})
m.eval()
eng = m.engine(dev)
if len(sys.argv) > 1: eng.set_precision(sys.argv[1])
B = 512
xe = torch.randn(B, 32, 16, device=dev); xd = torch.randn(B, 15, 16, device=dev); out = torch.empty(B, 5, 16, device=dev)
for _ in range(20): eng.forward(xe, xd, out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(500): eng.forward(xe, xd, out)
e1.record(); torch.cuda.synchronize()
print(eng.last_path(), eng.precision(), round(e0.elapsed_time(e1) / 500, 4), "ms", float(out.double().sum()))
