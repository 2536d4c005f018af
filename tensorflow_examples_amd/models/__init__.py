"""Model zoo: reference models (linear regression, MNIST MLP) and north-star models
(MNIST softmax, LeNet-5, ResNet-CIFAR, word2vec, char-LSTM)."""
