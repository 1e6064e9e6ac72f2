"""Which HIP runtime does each load order bind (diagnostic)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
order = sys.argv[1]
def maps():
    return sorted({l.split()[-1] for l in open('/proc/self/maps') if 'amdhip64' in l or 'hsa-runtime' in l or 'rccl' in l})
if order == 'torch_first':
    import torch
    print('torch count', torch.cuda.device_count()); x = torch.ones(4, device='cuda'); print('torch ok', x.sum().item())
    from fugu_amd import native
    print('native count', native.device_count()); ctx = native.Context((0,)); print('native ctx ok')
elif order == 'native_first':
    from fugu_amd import native
    print('native count', native.device_count()); ctx = native.Context((0,)); print('native ctx ok')
    import torch
    print('torch count', torch.cuda.device_count()); x = torch.ones(4, device='cuda'); print('torch ok', x.sum().item())
print(maps())
