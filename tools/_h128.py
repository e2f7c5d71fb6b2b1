import time, torch, sys
sys.path.insert(0, '../tests')
from conftest import code_path
from ldpc_neural_decoder.models import create_message_gnn_decoder
from ldpc_neural_decoder.utils import expand_base_matrix, load_base_matrix
base = load_base_matrix(code_path(32)); H = expand_base_matrix(base, 32)
for hid, B in ((64, 2048), (96, 1024), (128, 1024), (256, 256), (320, 64)):
    dec, conv = create_message_gnn_decoder(H, num_iterations=10, hidden_dim=hid, base_graph=base, Z=32)
    dec = dec.cuda()
    types = conv.get_message_types(base, 32)
    llr = (torch.randn(B, H.shape[1]) * 2 + 1).cuda()
    args = (llr, conv.message_to_var_index(), types, conv.var_to_check_adjacency, conv.check_to_var_adjacency)
    with torch.no_grad():
        dec(*args); torch.cuda.synchronize()
        t = time.perf_counter(); dec(*args); torch.cuda.synchronize(); dt = time.perf_counter() - t
    print(f"H={hid} B={B}: {dt*1e3:.1f} ms, {B/dt:.0f} cw/s", flush=True)
