import sys, torch, numpy as np
sys.path.insert(0, '.')
from perseus_amd import _lib, synth
from perseus_amd.detector import KeypointCNN
L=_lib.lib()
m=KeypointCNN(num_channels=4); m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k,v in synth.synthetic_state_dict(0).items()})
x=torch.from_numpy(synth.synthetic_frames(0,64)).cuda()
for v in [0,5,6,3]:
    for l in range(5): L.pa_debug_set_variant(l, v)
    prof,y=m.profile(x)
    y2 = torch.full_like(y, float('nan'))
    rc = L.pa_detector_forward(m._handle, x.data_ptr(), 64, y2.data_ptr(), _lib.stream_of(x.device))
    torch.cuda.synchronize()
    print(v, rc, L.pa_last_error(), [round(ms*1e3,1) for n,ms in prof][:6], torch.isnan(y2).any().item(), (y2-y).abs().max().item())
