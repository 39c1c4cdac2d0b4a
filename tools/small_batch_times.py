import sys, torch, numpy as np
sys.path.insert(0, ".")
from perseus_amd import synth
from perseus_amd.detector import KeypointCNN
m = KeypointCNN(num_channels=4)
m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
for B in (1, 3):
    x = torch.from_numpy(synth.synthetic_frames(0, B)).cuda()
    m(x)
    r = [m.time_launch(x, i, 20) for i in range(18)]
    print(B, round(sum(t for _, t in r) * 1e3, 1), [(n, round(t * 1e3, 1)) for n, t in r])
