'''

a very simple example - to demonstrate a working example on tensorflow_examples_amd
(MI355X-native re-implementation of R/simple/simple.py: linear regression W*x + b,
sum-of-squares loss, gradient descent lr 0.01, 1005 steps, same output line).

The model and loss are built from the framework's differentiable ops and the gradients come from
its autodiff (the reference's ``GradientDescentOptimizer(0.01).minimize(loss)``,
R/simple/simple.py:22-23): ``ops.scale_shift`` (W * x + b) -> ``ops.sum_squared_error`` ->
``loss.backward()`` accumulates dW, db into the flat gradient buffer -> the fused SGD kernel applies
them.  ``--device cuda`` runs every step on HIP kernels (elementwise.hip + optim.hip).

'''
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tensorflow_examples_amd import ops  # noqa: E402
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


def loss_of(x, y):
    linear_model = ops.scale_shift(x, W, b)                # linear_model = W * x + b
    return ops.sum_squared_error(linear_model, y)          # loss = reduce_sum(square(linear_model - y))


optimizer = GradientDescentOptimizer(store, 0.01)          # tf.train.GradientDescentOptimizer(0.01)
x = torch.tensor(x_train, dtype=torch.float32, device=store.device)   # feed x: x_train
y = torch.tensor(y_train, dtype=torch.float32, device=store.device)   # feed y: y_train
for i in range(args.steps):
    store.zero_grad()                                      # sess.run(train, {x: x_train, y: y_train}):
    loss_of(x, y).backward()                               #   gradients by the framework's autodiff
    optimizer.apply_gradients()                            #   ApplyGradientDescent on W and b

with torch.no_grad():
    curr_loss = loss_of(x, y)
curr_W, curr_b, curr_loss = W.master.cpu().numpy(), b.master.cpu().numpy(), np.float32(curr_loss.cpu().numpy())
print("W: %s b: %s loss %s" % (curr_W, curr_b, curr_loss))
