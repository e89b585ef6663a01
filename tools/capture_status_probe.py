"""Does a stream that joined a capture (wait_stream on the capturing stream) report itself capturing?
(torch's ProcessGroupNCCL skips its watchdog for collectives issued on capturing streams.)"""
import torch

torch.cuda.init()
side = torch.cuda.Stream()
x = torch.zeros(16, device="cuda")
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    cur = torch.cuda.current_stream()
    print("origin capturing:", torch.cuda.is_current_stream_capturing(), flush=True)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        print("joined side stream capturing:", torch.cuda.is_current_stream_capturing(), flush=True)
        x.add_(1)
    cur.wait_stream(side)
g.replay()
torch.cuda.synchronize()
print("after replay", float(x[0]))
