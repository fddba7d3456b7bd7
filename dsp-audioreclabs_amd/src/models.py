"""Drop-in for the reference's src/models.py (classifiers) on MI355X.

``TraditionalClassifier('knn')`` (models.py:18-72) -- the classifier on the north-star path --
runs the exact k-NN kernel (csrc/knn.hip, dsp_knn_classify): the same neighbours, distances and
majority vote as scikit-learn's KNeighborsClassifier(n_neighbors=k) (kd_tree, Euclidean,
uniform weights, scipy.stats.mode: smallest label on ties).  The other classifier types of the
reference (naive_bayes, decision_tree, svm) are not part of the accelerated path (SURVEY.md §8,
DESIGN.md §7); they keep the reference's scikit-learn models so a caller switching over loses
nothing.  The reference's MLP (models.py:77-221, PyTorch training) is out of scope.
"""
import numpy as np

from .pipeline import KnnIndex


class TraditionalClassifier:
    """models.py:18-72: fit / predict / evaluate with the reference's hyper-parameters."""

    def __init__(self, classifier_type='knn', **kwargs):
        self.classifier_type = classifier_type
        if classifier_type == 'knn':
            self.n_neighbors = int(kwargs.get('n_neighbors', 3))
            self.model = None
        elif classifier_type == 'naive_bayes':
            from sklearn.naive_bayes import GaussianNB
            self.model = GaussianNB()
        elif classifier_type == 'decision_tree':
            from sklearn.tree import DecisionTreeClassifier
            self.model = DecisionTreeClassifier(max_depth=kwargs.get('max_depth', None), random_state=42)
        elif classifier_type == 'svm':
            from sklearn.svm import SVC
            self.model = SVC(C=kwargs.get('C', 1.0), kernel=kwargs.get('kernel', 'rbf'), random_state=42)
        else:
            raise ValueError(f"不支持的分类器类型: {classifier_type}")

    def fit(self, X_train, y_train):
        if self.classifier_type != 'knn':
            self.model.fit(X_train, y_train)
            return self
        X = np.asarray(X_train, dtype=np.float64)
        y = np.asarray(y_train)
        if len(X) < self.n_neighbors:
            raise ValueError("Expected n_neighbors <= n_samples_fit, but n_neighbors = %d, n_samples_fit = %d"
                             % (self.n_neighbors, len(X)))
        # classes_ sorted as in scikit-learn; the vote's smallest-index tie break is then the
        # smallest label (scipy.stats.mode)
        self.classes_, codes = np.unique(y, return_inverse=True)
        # the reference set on the device, converted for the screen at the first query and kept
        self._index = KnnIndex(X, codes.astype(np.int32), self.n_neighbors, n_classes=len(self.classes_))
        return self

    def kneighbors(self, X_test):
        """(distances, indices) [n, k] like KNeighborsClassifier.kneighbors(X_test)."""
        idx, dist, _ = self._index.query(np.asarray(X_test, dtype=np.float64))
        return dist.cpu().numpy(), idx.cpu().numpy().astype(np.int64)

    def predict(self, X_test):
        if self.classifier_type != 'knn':
            return self.model.predict(X_test)
        _, _, pred = self._index.query(np.asarray(X_test, dtype=np.float64))
        return self.classes_[pred.cpu().numpy()]

    def evaluate(self, X_test, y_test):
        from sklearn.metrics import accuracy_score, classification_report, confusion_matrix
        y_pred = self.predict(X_test)
        return {
            'accuracy': accuracy_score(y_test, y_pred),
            'predictions': y_pred,
            'classification_report': classification_report(y_test, y_pred, output_dict=True, zero_division=0),
            'confusion_matrix': confusion_matrix(y_test, y_pred),
        }


def create_classifier(classifier_type, **kwargs):
    """models.py:226-246."""
    if classifier_type in ['knn', 'naive_bayes', 'decision_tree', 'svm']:
        return TraditionalClassifier(classifier_type, **kwargs)
    if classifier_type == 'mlp':
        raise NotImplementedError("the MLP classifier (models.py:77-221) is outside the accelerated path")
    raise ValueError(f"不支持的分类器类型: {classifier_type}")
