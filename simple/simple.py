'''

a very simple example - to demonstrate a working example on tensorflow_examples_amd
(MI355X-native re-implementation of R/simple/simple.py: linear regression W*x + b,
sum-of-squares loss, gradient descent lr 0.01, 1005 steps, same output line).

'''
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tensorflow_examples_amd.optim import GradientDescentOptimizer  # noqa: E402
from tensorflow_examples_amd.variables import Constant, VariableStore  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--device", default="cpu", help="cpu (default, like the reference) or cuda")
ap.add_argument("--steps", type=int, default=1005)
args = ap.parse_args()

store = VariableStore(device=args.device, compute_dtype=torch.float32)
W = store.variable([1], Constant(.3), name="Variable")     # tf.Variable([.3], tf.float32)
b = store.variable([1], Constant(-.3), name="Variable")    # tf.Variable([-.3], tf.float32) -> "Variable_1"
store.finalize()                                           # global_variables_initializer + sess.run(init)

x_train = [1, 2, 3, 4]
y_train = [0, -1, -2, -3]


def model_loss(x, y):
    # linear_model = W * x + b ; loss = reduce_sum(square(linear_model - y))
    return ((W.master * x + b.master - y) ** 2).sum()


def grads(x, y):
    # TF1 gradient graph of the loss above: d/dr = 2r, dW = sum(2r * x), db = sum(2r)
    r = W.master * x + b.master - y
    g = 2.0 * r
    W.grad.copy_(torch.sum(g * x).reshape(1))
    b.grad.copy_(torch.sum(g).reshape(1))


optimizer = GradientDescentOptimizer(store, 0.01)          # tf.train.GradientDescentOptimizer(0.01)
x = torch.tensor(x_train, dtype=torch.float32, device=store.device)
y = torch.tensor(y_train, dtype=torch.float32, device=store.device)
for i in range(args.steps):
    grads(x, y)                                            # sess.run(train, {x: x_train, y: y_train})
    optimizer.apply_gradients()

curr_W, curr_b, curr_loss = (W.master.cpu().numpy(), b.master.cpu().numpy(),
                             np.float32(model_loss(x, y).cpu().numpy()))
print("W: %s b: %s loss %s" % (curr_W, curr_b, curr_loss))
