import cProfile, pstats, sys, time, torch
sys.path.insert(0, '.')
from docker_dist_nn_amd import MLPSpec
from docker_dist_nn_amd.engine import OptimConfig, Trainer
from docker_dist_nn_amd.data import DeviceDataset, synthetic_mnist
dev = torch.device('cuda')
spec = MLPSpec.parse('784-128-64-10')
tr = Trainer(spec, micro_batch=64, num_micro=1, optim=OptimConfig(name='adam', lr=1e-3), device=dev)
x, y = synthetic_mnist(60000, seed=1)
data = DeviceDataset(x, y, 64, dev, kp=tr.stages[0].x_in.shape[1])
def one(i):
    xb, yb = data.batch(i)
    tr.set_batch(xb, yb, zero_copy=True)
    tr.step()
for i in range(50): one(i)
torch.cuda.synchronize()
t = time.perf_counter()
for i in range(500): one(i)
h = time.perf_counter() - t
torch.cuda.synchronize()
print("host us/step", h / 500 * 1e6, "total us/step", (time.perf_counter() - t) / 500 * 1e6)
pr = cProfile.Profile(); pr.enable()
for i in range(500): one(i)
pr.disable(); torch.cuda.synchronize()
pstats.Stats(pr).sort_stats('tottime').print_stats(14)
