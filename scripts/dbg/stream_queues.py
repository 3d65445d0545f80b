"""Which hardware queue (rocprofv3 Queue_Id) each kind of torch stream gets:
run under rocprofv3 --kernel-trace; one tiny kernel per stream, in creation
order, tagged by its element count (65536 (k + 1)) so the trace names the stream."""
import torch

dev = torch.device("cuda", 0)
streams = [("current", torch.cuda.current_stream(dev))]
streams += [(f"pool{k}", torch.cuda.Stream(dev)) for k in range(6)]
streams += [(f"high{k}", torch.cuda.Stream(dev, priority=-1)) for k in range(3)]
streams += [(f"ext{k}", torch.cuda.ExternalStream(torch.cuda.Stream(dev).cuda_stream)) for k in range(1)]
xs = []
for k, (name, s) in enumerate(streams):
    with torch.cuda.stream(s):
        x = torch.zeros(65536 * (k + 1), device=dev)  # grid size names the stream in the trace
        x.add_(1.0)
        xs.append(x)
    torch.cuda.synchronize()
    print(k, name, hex(s.cuda_stream), s.priority)
torch.cuda.synchronize()
