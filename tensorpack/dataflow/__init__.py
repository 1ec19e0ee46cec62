"""``tensorpack.dataflow`` serializer names for the driver's ``serializer=`` argument
(train_concap_struc.py:330, :347).  The storage engine itself is outside the hot path
(SURVEY.md §2): ``load`` / ``save`` raise with the conversion route instead of silently reading nothing."""


class _Serializer(object):
    @staticmethod
    def save(df, path):
        raise NotImplementedError("tensorpack LMDB containers are not written by the MI355X build; use "
                                  "k3m_amd.loaders.write_records")

    @staticmethod
    def load(path, shuffle=True):
        raise NotImplementedError("tensorpack LMDB containers are not read by the MI355X build; convert the records "
                                  "with k3m_amd.loaders.write_records (ConceptCapLoaderTrain_struc reads that)")


class LMDBSerializer(_Serializer):
    pass


class NumpySerializer(_Serializer):
    pass
